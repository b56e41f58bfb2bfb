"""ctypes binding of libvideoprism_hip.so (C-ABI declared in include/videoprism_hip.h).

There is no fallback: if the library is missing or cannot be loaded, every entry point
raises NativeLibraryError.  Device memory is passed as raw pointers of PyTorch-ROCm
tensors; streams as hipStream_t handles of torch streams.
"""

from __future__ import annotations

import ctypes
import os
from ctypes import POINTER, c_char_p, c_float, c_int, c_int32, c_int64, c_size_t, c_void_p

_LIB_NAME = "libvideoprism_hip.so"
_LIB_PATH = os.path.join(os.path.dirname(os.path.abspath(__file__)), _LIB_NAME)
# tools' A/B library (`make -C videoprism-mlx_amd diag`): the product library plus ablation builds;
# loaded only when VP_DIAG_LIB=1 (tools/), never by the package's tests or the bench
_DIAG_LIB_PATH = os.path.join(os.path.dirname(os.path.abspath(__file__)), "libvideoprism_hip_diag.so")

VP_OK, VP_EINVAL, VP_ENOMEM, VP_EHIP, VP_ESTATE, VP_ENOTSUP, VP_ECOMM = range(7)
VP_F32, VP_BF16, VP_U8 = 0, 1, 2

EPI_STORE, EPI_GELU, EPI_RESID, EPI_POS, EPI_RESID_FFN = 0, 1, 2, 3, 4
# bf16 residual stream variants (bf16 resid / out; bf16 precision only)
EPI_RESID_BF16, EPI_POS_BF16, EPI_RESID_FFN_BF16 = 5, 6, 7
PERM_NONE, PERM_BTN_TO_BNT, PERM_BNT_TO_BTN = 0, 1, 2


class NativeLibraryError(RuntimeError):
    """libvideoprism_hip.so is missing or failed to load (no CPU fallback exists)."""


class VPError(RuntimeError):
    def __init__(self, code: int, msg: str):
        super().__init__(f"[vp status {code}] {msg}")
        self.code = code


class vp_config(ctypes.Structure):
    _fields_ = [
        ("patch_size", c_int32),
        ("pos_emb_t", c_int32),
        ("pos_emb_h", c_int32),
        ("pos_emb_w", c_int32),
        ("model_dim", c_int32),
        ("num_spatial_layers", c_int32),
        ("num_temporal_layers", c_int32),
        ("num_heads", c_int32),
        ("mlp_dim", c_int32),
        ("atten_logit_cap", c_float),
        ("fprop_dtype", c_int32),
    ]


class vp_clip_config(ctypes.Structure):
    _fields_ = [
        ("video", vp_config),
        ("num_auxiliary_layers", c_int32),
        ("vocabulary_size", c_int32),
        ("num_unimodal_layers", c_int32),
        ("enable_causal_atten", c_int32),
    ]


# name -> (restype, argtypes)
_SIGNATURES = {
    "vp_last_error": (c_char_p, []),
    "vp_abi_version": (c_int, []),
    "vp_create": (c_int, [POINTER(vp_config), c_int, POINTER(c_void_p)]),
    "vp_destroy": (c_int, [c_void_p]),
    "vp_set_param": (c_int, [c_void_p, c_char_p, c_void_p, POINTER(c_int64), c_int]),
    "vp_param_count": (c_int, [c_void_p, POINTER(c_int)]),
    "vp_param_name": (c_int, [c_void_p, c_int, POINTER(c_char_p)]),
    "vp_finalize": (c_int, [c_void_p]),
    "vp_prepare_geometry": (c_int, [c_void_p, c_int64, c_int64]),
    "vp_prepare_frames": (c_int, [c_void_p, c_int64]),
    "vp_workspace_bytes": (c_int, [c_void_p, c_int64, c_int64, c_int64, c_int64, POINTER(c_size_t)]),
    "vp_forward": (c_int, [c_void_p, c_void_p, c_int, c_int64, c_int64, c_int64, c_int64, c_void_p,
                           c_void_p, c_int, c_void_p, c_void_p, c_size_t, c_void_p]),
    "vp_profile_enable": (c_int, [c_void_p, c_int]),
    "vp_profile_read": (c_int, [c_void_p, c_int, POINTER(ctypes.c_double), POINTER(ctypes.c_double),
                                POINTER(ctypes.c_double), POINTER(c_int64)]),
    "vp_profile_set_mask": (c_int, [c_void_p, ctypes.c_uint32]),
    "vp_profile_class_count": (c_int, []),
    "vp_profile_class_name": (c_int, [c_int, POINTER(c_char_p)]),
    "vp_profile_kernel_name": (c_int, [c_void_p, c_int, POINTER(c_char_p)]),
    # multi-GPU: RCCL all-gather of pooled clip embeddings
    "vp_comm_id_bytes": (c_int, []),
    "vp_comm_unique_id": (c_int, [c_void_p, c_int64]),
    "vp_comm_init": (c_int, [c_void_p, c_int64, c_int, c_int, c_int, POINTER(c_void_p)]),
    "vp_comm_destroy": (c_int, [c_void_p]),
    "vp_allgather": (c_int, [c_void_p, c_void_p, c_void_p, c_int64, c_int, c_void_p]),
    "vp_op_gemm": (c_int, [c_int, c_int, c_void_p, c_int64, c_void_p, c_int64, c_int64, c_int64,
                           c_int64, c_void_p, c_int64, c_void_p, c_void_p, c_int64, c_void_p,
                           c_int64, c_void_p, c_void_p]),
    "vp_op_attention": (c_int, [c_int, c_void_p, c_void_p, c_int64, c_int64, c_int64, c_float,
                                c_void_p, c_void_p]),
    "vp_op_layernorm": (c_int, [c_void_p, c_int, c_int64, c_int64, c_void_p, c_void_p, c_void_p,
                                c_int, c_int, c_int64, c_int64, c_void_p, c_void_p]),
    "vp_op_patchify": (c_int, [c_void_p, c_int, c_void_p, c_int, c_int64, c_int64, c_int64, c_int64,
                               c_int64, c_int64, c_void_p]),
    "vp_op_pool_l2": (c_int, [c_void_p, c_int, c_int64, c_int64, c_int64, c_void_p, c_void_p]),
    "vp_op_attention_masked": (c_int, [c_int, c_void_p, c_void_p, c_int64, c_int64, c_int64, c_float,
                                       c_void_p, c_int, c_void_p]),
    "vp_op_similarity": (c_int, [c_void_p, c_void_p, c_int64, c_int64, c_int64, c_void_p, c_void_p]),
    # LvT video-text model (FactorizedVideoCLIP)
    "vp_clip_create": (c_int, [POINTER(vp_clip_config), c_int, POINTER(c_void_p)]),
    "vp_clip_destroy": (c_int, [c_void_p]),
    "vp_clip_set_param": (c_int, [c_void_p, c_char_p, c_void_p, POINTER(c_int64), c_int]),
    "vp_clip_param_count": (c_int, [c_void_p, POINTER(c_int)]),
    "vp_clip_param_name": (c_int, [c_void_p, c_int, POINTER(c_char_p)]),
    "vp_clip_finalize": (c_int, [c_void_p]),
    "vp_clip_video_handle": (c_int, [c_void_p, POINTER(c_void_p)]),
    "vp_clip_video_workspace_bytes": (c_int, [c_void_p, c_int64, c_int64, c_int64, c_int64,
                                              POINTER(c_size_t)]),
    "vp_clip_encode_video": (c_int, [c_void_p, c_void_p, c_int, c_int64, c_int64, c_int64, c_int64,
                                     c_void_p, c_int, c_void_p, c_void_p, c_void_p, c_void_p, c_int,
                                     c_void_p, c_size_t, c_void_p]),
    # FactorizedVideoClassifier
    "vp_classifier_create": (c_int, [POINTER(vp_config), c_int, c_int, POINTER(c_void_p)]),
    "vp_classifier_destroy": (c_int, [c_void_p]),
    "vp_classifier_set_param": (c_int, [c_void_p, c_char_p, c_void_p, POINTER(c_int64), c_int]),
    "vp_classifier_param_count": (c_int, [c_void_p, POINTER(c_int)]),
    "vp_classifier_param_name": (c_int, [c_void_p, c_int, POINTER(c_char_p)]),
    "vp_classifier_finalize": (c_int, [c_void_p]),
    "vp_classifier_video_handle": (c_int, [c_void_p, POINTER(c_void_p)]),
    "vp_classifier_workspace_bytes": (c_int, [c_void_p, c_int64, c_int64, c_int64, c_int64,
                                              POINTER(c_size_t)]),
    "vp_classifier_forward": (c_int, [c_void_p, c_void_p, c_int, c_int64, c_int64, c_int64, c_int64,
                                      c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_int,
                                      c_void_p, c_size_t, c_void_p]),
    "vp_clip_text_workspace_bytes": (c_int, [c_void_p, c_int64, c_int64, POINTER(c_size_t)]),
    "vp_clip_encode_text": (c_int, [c_void_p, c_void_p, c_void_p, c_int64, c_int64, c_int, c_void_p,
                                    c_void_p, c_size_t, c_void_p]),
    # not in the public header: named-kernel GEMM for A/B tests and tools/gemm_bench.py
    "vp_dev_gemm_kernel": (c_int, [c_int, c_int, c_void_p, c_void_p, c_int64, c_int64, c_int64,
                                   c_void_p, c_void_p, c_void_p, c_void_p, c_int64, c_void_p,
                                   c_void_p]),
    "vp_dev_gemm_ln": (c_int, [c_int, c_void_p, c_void_p, c_int64, c_int64, c_int64, c_void_p,
                               c_void_p, c_void_p, c_void_p, c_int64, c_void_p, c_void_p,
                               c_void_p, c_void_p, c_void_p]),
    "vp_dev_ln_stats": (c_int, [c_int, c_void_p, c_int64, c_int64, c_void_p, c_void_p]),
    "vp_dev_patch_embed": (c_int, [c_void_p, c_int64, c_int64, c_void_p, c_int64, c_void_p, c_void_p, c_void_p,
                                   c_void_p]),
    "vp_dev_attention_spatial_blk": (c_int, [c_void_p, c_void_p, c_int64, c_int64, c_float, c_void_p, c_void_p]),
    "vp_dev_gemm_tattn": (c_int, [c_int, c_void_p, c_void_p, c_int64, c_int64, c_void_p, c_void_p, c_void_p,
                                  c_void_p, c_void_p, c_int64, c_float, c_void_p]),
}
# diag library only (ablation builds for tools/)
_DIAG_SIGNATURES = {
    "vp_dev_gemm_f32_var": (c_int, [c_int, c_int, c_int, c_void_p, c_void_p, c_int64, c_int64, c_int64, c_void_p,
                                    c_void_p, c_void_p]),
    "vp_dev_attention_long_var": (c_int, [c_int, c_void_p, c_void_p, c_int64, c_int64, c_int64, c_float, c_void_p]),
    "vp_dev_gemm_tattn_abl": (c_int, [c_int, c_int, c_void_p, c_void_p, c_int64, c_int64, c_void_p, c_void_p,
                                      c_void_p, c_void_p, c_void_p, c_int64, c_float, c_void_p]),
    "vp_dev_gemm_w4_abl": (c_int, [c_int, c_int, c_void_p, c_void_p, c_int64, c_int64, c_int64, c_void_p,
                                   c_void_p, c_void_p]),
    "vp_dev_gemm_ffn1_abl": (c_int, [c_int, c_void_p, c_void_p, c_int64, c_int64, c_int64, c_void_p, c_void_p,
                                     c_void_p, c_void_p, c_void_p]),
    "vp_dev_gemm_ffn2_abl": (c_int, [c_int, c_void_p, c_void_p, c_int64, c_int64, c_int64, c_void_p, c_void_p,
                                     c_void_p, c_void_p]),
}

_lib = None


def _diag() -> bool:
    return os.environ.get("VP_DIAG_LIB", "0") == "1"


def library_path() -> str:
    return _DIAG_LIB_PATH if _diag() else _LIB_PATH


def load() -> ctypes.CDLL:
    """Loads (once) and returns the library; raises NativeLibraryError if unavailable."""
    global _lib
    if _lib is not None:
        return _lib
    path = library_path()
    if not os.path.exists(path):
        raise NativeLibraryError(
            f"{path} not found: build it with `make -C videoprism-mlx_amd` "
            "(or __graft_entry__.build()); there is no CPU fallback.")
    try:
        import torch  # noqa: F401  (HIP runtime / RCCL of the process: torch's, loaded first)
    except ImportError:  # pragma: no cover
        pass
    try:
        lib = ctypes.CDLL(path)
    except OSError as e:
        raise NativeLibraryError(f"failed to load {path}: {e}") from e
    sigs = dict(_SIGNATURES, **(_DIAG_SIGNATURES if _diag() else {}))
    for name, (res, args) in sigs.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    _lib = lib
    return lib


def exported_symbols():
    return list(_SIGNATURES)


def check(rc: int) -> None:
    if rc != VP_OK:
        msg = load().vp_last_error().decode("utf-8", "replace")
        if rc in (VP_EINVAL,):
            raise ValueError(msg)
        if rc == VP_ENOTSUP:
            raise NotImplementedError(msg)
        raise VPError(rc, msg)


def call(name: str, *args) -> None:
    fn = getattr(load(), name)
    # an undeclared signature would pass Python ints as 32-bit c_int: a device pointer truncated that way
    # is an illegal address on the GPU, so every entry point called here must be declared
    if getattr(fn, "argtypes", None) is None:
        raise TypeError(f"{name}: no ctypes signature declared in _native.py")
    check(fn(*args))


# ---------------------------------------------------------------------------------------
# torch-tensor helpers for the op-level entry points (used by kernel parity tests)
# ---------------------------------------------------------------------------------------
def _ptr(t):
    return None if t is None else c_void_p(t.data_ptr())


def _stream(stream=None):
    import torch
    s = stream if stream is not None else torch.cuda.current_stream()
    return c_void_p(s.cuda_stream)


def _prec(t):
    import torch
    if t.dtype == torch.bfloat16:
        return VP_BF16
    if t.dtype == torch.float32:
        return VP_F32
    if t.dtype == torch.uint8:
        return VP_U8
    raise TypeError(f"unsupported dtype {t.dtype}")


def op_gemm(a, w, bias, epilogue=EPI_STORE, out=None, resid=None, pos=None, rowpad=None,
            stream=None):
    """out = epilogue(a @ w.T + bias); a [M,K], w [N,K] (bf16 or fp32), bias fp32 [N]."""
    import torch
    M, K = a.shape
    N = w.shape[0]
    if out is None:
        odt = (a.dtype if epilogue in (EPI_STORE, EPI_GELU) else
               torch.bfloat16 if epilogue >= EPI_RESID_BF16 else torch.float32)
        out = torch.empty((M, N), dtype=odt, device=a.device)
    call("vp_op_gemm", _prec(a), epilogue, _ptr(a), a.stride(0), _ptr(w), w.stride(0), M, N, K,
         _ptr(out), out.stride(0), _ptr(bias), _ptr(resid),
         resid.stride(0) if resid is not None else 0, _ptr(pos),
         pos.shape[0] if pos is not None else 0, _ptr(rowpad), _stream(stream))
    return out


def dev_gemm_kernel(which, a, w, bias, epilogue, out, resid=None, pos=None, rowpad=None,
                    stream=None):
    """bf16 GEMM through one named kernel (4 = 4-wave, 8 = 8-wave); out/resid contiguous."""
    M, K = a.shape
    N = w.shape[0]
    call("vp_dev_gemm_kernel", which, epilogue, _ptr(a), _ptr(w), M, N, K, _ptr(out), _ptr(bias),
         _ptr(resid), _ptr(pos), pos.shape[0] if pos is not None else 0, _ptr(rowpad),
         _stream(stream))
    return out


EPI_BF16_LN, EPI_GELU_LN, EPI_RESID_BF16_ST, EPI_RESID_FFN_BF16_ST, EPI_POS_BF16_ST = 8, 9, 10, 11, 12
# the FFN pair over the row-blocked hidden activation [M/16][F/32][16][32] (vp_kernels.h EPI_*_BLK)
EPI_GELU_LN_BLK, EPI_RESID_FFN_BF16_ST_BLK, EPI_RESID_FFN_BF16_BLK, EPI_BF16_LN_BLK = 16, 17, 18, 19


def ffn1_blk_rows(F):
    """Row order of W1 / b' / c for EPI_GELU_LN_BLK (vp_internal.h pack_stack): packed row r holds
    natural row src[r] -- within each 32-row group, row 16 h + 4 g + i holds column 8 g + 4 h + i."""
    import numpy as np
    r = np.arange(F)
    w = r & 31
    return (r & ~31) + 8 * ((w >> 2) & 3) + 4 * (w >> 4) + (w & 3)


def to_row_blocked(h):
    """[M, F] row-major -> the [M/16][F/32][16][32] blocked layout, flattened back to [M, F] storage."""
    M, F = h.shape
    return h.reshape(M // 16, 16, F // 32, 32).permute(0, 2, 1, 3).reshape(M, F)


def dev_gemm_ln(a, w, bias, epilogue, out, resid=None, pos=None, rowpad=None, ln_rs=None,
                ln_c=None, st_part=None, stream=None):
    """bf16 w4 GEMM with a GEMM-folded LayerNorm epilogue (8, 9) or a row-statistics
    epilogue (10..12); all tensors contiguous on the device."""
    M, K = a.shape
    N = w.shape[0]
    call("vp_dev_gemm_ln", epilogue, _ptr(a), _ptr(w), M, N, K, _ptr(out), _ptr(bias), _ptr(resid),
         _ptr(pos), pos.shape[0] if pos is not None else 0, _ptr(rowpad), _ptr(ln_rs), _ptr(ln_c),
         _ptr(st_part), _stream(stream))
    return out


def dev_gemm_w4_abl(a, w, bias, out, abl, s3=False, stream=None):
    """Diag library only: an ablation build of the product 4-wave GEMM (EPI_BF16; abl 2 = no
    ds_reads, 4 = no staging loads, 8 = no epilogue) -- timing only, results garbage."""
    M, K = a.shape
    N = w.shape[0]
    call("vp_dev_gemm_w4_abl", abl, 1 if s3 else 0, _ptr(a), _ptr(w), M, N, K, _ptr(out), _ptr(bias),
         _stream(stream))
    return out


def dev_gemm_tattn(which, a, w, bias, ln_rs, ln_c, out, heads, cap, p=None, stream=None):
    """The fused temporal attention's launches: which 0 (w = [q_h | k_h] rows) -> P in `out`,
    which 1 (w = v rows, p = P) -> O [M, D] in `out`; all tensors contiguous on the device."""
    M, K = a.shape
    call("vp_dev_gemm_tattn", which, _ptr(a), _ptr(w), M, K, _ptr(out), _ptr(bias), _ptr(ln_rs), _ptr(ln_c),
         _ptr(p), heads, float(cap), _stream(stream))
    return out


def video_patch_w(k, P):
    """The fused patch embedding's weight layout (vp_kernels.h video_patch_k; packed the same way by
    vp_finalize): k [P*P*3, N] (the patch kernel) -> [N, 64 P]: patch pixel row py is K-tile py, read as
    cpr = ceil(3P/8) chunks of 8 values at value offsets min(8 j, 3P - 8) in slots j < cpr (columns
    64 py + 8 j ..); zero where a row's last chunk overlaps its predecessor and in the slots j >= cpr."""
    import torch
    cpr = (3 * P + 7) // 8
    kv = 64 * P
    out = torch.zeros(k.shape[1], kv, dtype=k.dtype)
    for py in range(P):
        for cr in range(cpr):
            vo = min(8 * cr, 3 * P - 8)
            for e in range(8):
                v = vo + e
                if cr == cpr - 1 and v < 8 * (cpr - 1):
                    continue
                out[:, 64 * py + 8 * cr + e] = k[py * 3 * P + v]
    return out


def dev_patch_embed(video, P, wv, bias, pos, out, stream=None):
    """Fused patch embedding (EPI_POS_BF16) straight from bf16 frames [F, 16P, 16P, 3]."""
    frames = video.shape[0]
    call("vp_dev_patch_embed", _ptr(video), frames, P, _ptr(wv), wv.shape[0], _ptr(bias), _ptr(pos), _ptr(out),
         _stream(stream))
    return out


def dev_ln_stats(src, M, D, out, from_partials, stream=None):
    """(rstd, -mean*rstd) per row from partial statistics (from_partials) or bf16 rows."""
    call("vp_dev_ln_stats", 0 if from_partials else 1, _ptr(src), M, D, _ptr(out), _stream(stream))
    return out


def op_attention(qkv, num_seq, S, heads, cap, key_pad=None, out=None, stream=None):
    import torch
    D = heads * 64
    if out is None:
        out = torch.empty((num_seq * S, D), dtype=qkv.dtype, device=qkv.device)
    call("vp_op_attention", _prec(qkv), _ptr(qkv), _ptr(out), num_seq, S, heads, float(cap),
         _ptr(key_pad), _stream(stream))
    return out


def op_attention_masked(qkv, num_seq, S, heads, cap, key_pad=None, causal=False, out=None,
                        stream=None):
    """Generic fp32-math attention with key paddings and the causal merge (text tower)."""
    import torch
    D = heads * 64
    if out is None:
        out = torch.empty((num_seq * S, D), dtype=qkv.dtype, device=qkv.device)
    call("vp_op_attention_masked", _prec(qkv), _ptr(qkv), _ptr(out), num_seq, S, heads, float(cap),
         _ptr(key_pad), 1 if causal else 0, _stream(stream))
    return out


def op_similarity(video_emb, text_emb, stream=None):
    """video_emb [B, D] . text_emb [Q, D]^T (fp32)."""
    import torch
    B, D = video_emb.shape
    Q = text_emb.shape[0]
    out = torch.empty((B, Q), dtype=torch.float32, device=video_emb.device)
    call("vp_op_similarity", _ptr(video_emb), _ptr(text_emb), B, Q, D, _ptr(out), _stream(stream))
    return out


def op_layernorm(x, gamma1p, beta, out_dtype=None, perm=PERM_NONE, T=1, Nsp=1, add=None,
                 stream=None):
    import torch
    rows, D = x.shape
    out_dtype = out_dtype or torch.float32
    out = torch.empty((rows, D), dtype=out_dtype, device=x.device)
    call("vp_op_layernorm", _ptr(x), _prec(x), rows, D, _ptr(gamma1p), _ptr(beta), _ptr(out),
         VP_BF16 if out_dtype == torch.bfloat16 else VP_F32, perm, T, Nsp, _ptr(add),
         _stream(stream))
    return out


def op_patchify(video, P, kpad, out_dtype=None, stream=None):
    import torch
    BT, H, W, C = video.shape
    out_dtype = out_dtype or video.dtype
    out = torch.empty((BT * (H // P) * (W // P), kpad), dtype=out_dtype, device=video.device)
    call("vp_op_patchify", _ptr(video), _prec(video), _ptr(out),
         VP_BF16 if out_dtype == torch.bfloat16 else VP_F32, BT, H, W, C, P, kpad, _stream(stream))
    return out


def op_pool_l2(emb, stream=None):
    import torch
    B, L, D = emb.shape
    out = torch.empty((B, D), dtype=torch.float32, device=emb.device)
    call("vp_op_pool_l2", _ptr(emb), _prec(emb), B, L, D, _ptr(out), _stream(stream))
    return out


def source_fingerprint() -> str:
    """sha256 over the product library's sources (the Makefile's SRC list, csrc/ headers and
    include/): bench.py only quotes PMC traffic measured on a build of exactly these sources.
    Files only the tools' diag library compiles (DIAG_SRC) do not count."""
    import hashlib
    import re
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    csrc = os.path.join(root, "csrc")
    with open(os.path.join(root, "Makefile")) as fh:
        m = re.search(r"^SRC\s*:=\s*(.+)$", fh.read(), re.M)
    product = {os.path.basename(f) for f in m.group(1).split()} if m else None
    files = []
    for d in (csrc, os.path.join(os.path.dirname(root), "include")):
        if os.path.isdir(d):
            files += sorted(os.path.join(d, f) for f in os.listdir(d)
                            if f.endswith(".h") or (f.endswith((".hip", ".cpp")) and
                                                    (product is None or f in product)))
    h = hashlib.sha256()
    for f in files:
        h.update(os.path.basename(f).encode())
        with open(f, "rb") as fh:
            h.update(fh.read())
    return h.hexdigest()[:16]


def kernel_short_name(symbol: str) -> str:
    """'void vp::(anonymous namespace)::gemm_bf16_w4_kernel<9, 512, 0>(...)' ->
    'gemm_bf16_w4_kernel<9, 512, 0>' (the same key tools/pmc_summary.py gives rocprof's names)."""
    import re
    m = re.search(r"(\w+_kernel\w*)<([^>]*)>", symbol)
    if m:
        return f"{m.group(1)}<{m.group(2)}>"
    m = re.search(r"(\w+_kernel\w*)\b", symbol)
    return m.group(1) if m else symbol


def profile_kernel_name(handle, cls_name: str) -> str:
    """Short symbol of the kernel last launched for profiler class `cls_name` on `handle`."""
    lib = load()
    for i in range(lib.vp_profile_class_count()):
        n = ctypes.c_char_p()
        call("vp_profile_class_name", i, ctypes.byref(n))
        if n.value.decode() == cls_name:
            k = ctypes.c_char_p()
            call("vp_profile_kernel_name", handle, i, ctypes.byref(k))
            return kernel_short_name(k.value.decode()) if k.value else ""
    return ""
