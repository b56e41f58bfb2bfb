"""The MFMA rates this GPU sustains for the fp32 path's instructions beside the bf16 GEMMs' one
(tools/peak/mfma_peak.hip: every CU, one wave per SIMD, back-to-back MFMAs from registers on random
operands, in-kernel clock): v_mfma_f32_16x16x4_f32 (the fp32 GEMMs, gemm_f32.hip) and
v_mfma_f32_32x32x2_f32 (the fp32 attention, attn_f32_mfma_kernel).  Measurement only."""
import ctypes
import os

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    lib = ctypes.CDLL(os.path.join(ROOT, "tools", "peak", "libmfma_peak.so"))
    for shape, name in ((0, "v_mfma_f32_16x16x32_bf16"), (2, "v_mfma_f32_16x16x4_f32"), (3, "v_mfma_f32_32x32x2_f32")):
        best, med, clk, ms = (ctypes.c_double() for _ in range(4))
        iters = 4_000_000 if shape < 2 else 1_000_000
        rc = lib.mfma_peak_run(0, shape, iters, 3, ctypes.byref(best), ctypes.byref(med), ctypes.byref(clk),
                               ctypes.byref(ms))
        print(f"{name}: rc {rc} {med.value:.1f} TFLOP/s (best {best.value:.1f}) at {clk.value:.3f} GHz in-kernel, "
              f"{ms.value:.1f} ms per launch", flush=True)


if __name__ == "__main__":
    main()
