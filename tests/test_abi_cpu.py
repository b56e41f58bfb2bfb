"""The C-ABI library loads without a GPU and exports every symbol include/videoprism_hip.h
declares (no compute calls here)."""

import ctypes
import os
import re

import pytest

from videoprism import _native

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "videoprism_hip.h")


def header_symbols():
    text = open(HEADER).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(vp_\w+)\s*\(", text)))


def test_library_present_and_loads():
    assert os.path.exists(_native.library_path()), "build with __graft_entry__.build()"
    lib = _native.load()
    want = int(re.search(r"#define VP_ABI_VERSION (\d+)", open(HEADER).read()).group(1))
    assert lib.vp_abi_version() == want


def test_product_library_has_no_ablation_builds():
    """The A/B and ablation kernels live in the tools' diag library only (make diag): the product
    library exports no diag entry points and reads no kernel-selection environment switch."""
    lib = ctypes.CDLL(_native.library_path())
    for sym in ("vp_dev_gemm_diag", "vp_dev_attention_diag", "vp_dev_gemm_w4_abl", "vp_dev_gemm_ov",
                "vp_dev_gemm_w8b", "vp_dev_qkv_attention"):
        assert not hasattr(lib, sym), sym
    blob = open(_native.library_path(), "rb").read()
    assert b"VP_GEMM_KERNEL" not in blob and b"gemm_bf16_ov" not in blob and b"VP_NO_TATTN" not in blob
    assert b"gemm_bf16_w8b" not in blob and b"qkv_attn_spatial" not in blob
    # every 4-wave GEMM kernel in the product library is an ABL = 0 (production) instantiation
    import check_kernels
    names = [k[".name"] for k in check_kernels.kernels(_native.library_path())]
    w4 = [n for n in names if "gemm_bf16_w4_kernel" in n]
    abl = [re.search(r"gemm_bf16_w4_kernelILi\d+ELb[01]ELb[01]ELi(\d+)E", n) for n in w4]
    assert w4 and all(m is not None and m.group(1) == "0" for m in abl), w4


def test_comm_entry_points_without_a_gpu():
    """vp_comm_*: id size and argument checks (no RCCL call is made for bad arguments)."""
    lib = _native.load()
    assert lib.vp_comm_id_bytes() == 128
    h = ctypes.c_void_p()
    uid = (ctypes.c_uint8 * 128)()
    assert lib.vp_comm_init(uid, 128, 2, 5, 0, ctypes.byref(h)) == _native.VP_EINVAL
    assert lib.vp_comm_init(uid, 16, 2, 0, 0, ctypes.byref(h)) == _native.VP_EINVAL
    assert lib.vp_allgather(None, None, None, 1, 0, None) == _native.VP_EINVAL


def test_every_header_symbol_exported():
    syms = header_symbols()
    assert len(syms) >= 18
    lib = ctypes.CDLL(_native.library_path())
    missing = [s for s in syms if not hasattr(lib, s)]
    assert not missing, missing


def test_ctypes_bindings_cover_header():
    assert set(header_symbols()) <= set(_native.exported_symbols())


def test_header_compiles_as_c():
    import subprocess
    import tempfile
    src = '#include "videoprism_hip.h"\nint main(void){ vp_config c; (void)c; return VP_OK; }\n'
    with tempfile.TemporaryDirectory() as d:
        f = os.path.join(d, "t.c")
        open(f, "w").write(src)
        r = subprocess.run(["gcc", "-std=c99", "-Wall", "-Werror", "-I", os.path.dirname(HEADER),
                            "-c", f, "-o", os.path.join(d, "t.o")], capture_output=True, text=True)
        assert r.returncode == 0, r.stderr


def test_create_rejects_bad_configs_without_touching_a_gpu():
    lib = _native.load()
    h = ctypes.c_void_p()
    bad = _native.vp_config(patch_size=18, pos_emb_t=16, pos_emb_h=16, pos_emb_w=16, model_dim=768,
                            num_spatial_layers=12, num_temporal_layers=4, num_heads=16, mlp_dim=3072,
                            atten_logit_cap=50.0, fprop_dtype=1)   # dim_per_head 48
    rc = lib.vp_create(ctypes.byref(bad), 0, ctypes.byref(h))
    assert rc == _native.VP_ENOTSUP
    assert b"dim_per_head" in lib.vp_last_error()
    with pytest.raises(NotImplementedError):
        _native.check(rc)
    bad.num_heads = 0
    assert lib.vp_create(ctypes.byref(bad), 0, ctypes.byref(h)) == _native.VP_EINVAL


def test_null_arguments_are_einval():
    lib = _native.load()
    assert lib.vp_create(None, 0, None) == _native.VP_EINVAL
    assert lib.vp_finalize(None) == _native.VP_EINVAL
    assert lib.vp_forward(None, None, 0, 1, 1, 18, 18, None, None, 0, None, None, 0, None) == _native.VP_EINVAL
    assert lib.vp_op_attention(_native.VP_BF16, None, None, 1, 256, 12, 50.0, None, None) == _native.VP_EINVAL


def test_kernel_short_name_keys():
    """bench.py keys PMC traffic records (tools/pmc_summary.py) by the short kernel symbol: template names
    with a suffix after `_kernel` (gemm_f32_kernel2) keep their template arguments like the others."""
    from videoprism import _native
    assert _native.kernel_short_name("void vp::(anonymous namespace)::gemm_f32_kernel2<1>(float const*, long)") == \
        "gemm_f32_kernel2<1>"
    assert _native.kernel_short_name("void vp::(anonymous namespace)::gemm_bf16_w4_kernel<16, true, false, 0, false>"
                                     "(unsigned short const*)") == "gemm_bf16_w4_kernel<16, true, false, 0, false>"
    assert _native.kernel_short_name("void vp::(anonymous namespace)::layernorm_kernel(float const*)") == \
        "layernorm_kernel"
