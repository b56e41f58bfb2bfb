"""The build's kernel guards (tools/check_kernels.py, run by `make` after linking), on CPU:

* every kernel of the built product library has no scratch and no VGPR spills (the failure that
  faulted the round-3 experiment attn_long_pipe_kernel: inline-asm load destinations spilled while
  the loads were in flight);
* every inline-asm load with a VGPR destination either waits in its own statement or sits in a
  source whose device assembly is audited, and the audit of freshly generated assembly is clean;
* the guards do fire: an injected compiler copy / spill of an in-flight asm destination, and a
  kernel with a scratch array, are refused.
"""

import os
import re
import subprocess

import pytest

import check_kernels as ck
from videoprism import _native

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "videoprism-mlx_amd", "csrc")
HIPCC = "/opt/rocm/bin/hipcc"
FLAGS = ["-O3", "-std=c++17", "--offload-arch=gfx950", "-x", "hip"]


def _makefile_var(name):
    mk = open(os.path.join(ROOT, "videoprism-mlx_amd", "Makefile")).read()
    return re.search(rf"^{name} := (.*)$", mk, re.M).group(1).split()


def _hip_sources():
    srcs = [os.path.join(ROOT, "videoprism-mlx_amd", p) for p in _makefile_var("SRC") if p.endswith(".hip")]
    return srcs + [os.path.join(CSRC, h) for h in os.listdir(CSRC) if h.endswith(".h")]


@pytest.fixture(scope="module")
def audited_asm(tmp_path_factory):
    if not os.path.exists(HIPCC):
        pytest.skip("hipcc not available")
    out = tmp_path_factory.mktemp("asm")
    paths = []
    for rel in _makefile_var("ASM_AUDIT"):
        src = os.path.join(ROOT, "videoprism-mlx_amd", rel)
        dst = out / (os.path.splitext(os.path.basename(rel))[0] + ".s")
        subprocess.run([HIPCC, *FLAGS, "--cuda-device-only", "-S", src, "-o", str(dst)], check=True,
                       capture_output=True)
        paths.append(str(dst))
    return paths


def test_product_kernels_no_scratch_no_spills():
    lib = _native.library_path()
    assert os.path.exists(lib), "build with __graft_entry__.build()"
    ks = ck.kernels(lib)
    assert len(ks) > 50
    assert ck.resource_violations(lib) == []
    # the attention kernels with asm loads, by name, with their register budgets
    by = {k[".name"]: k for k in ks}
    spatial = [n for n in by if "attn_spatial_kernel" in n]
    long_ = [n for n in by if "attn_long_kernel" in n]
    # spatial: (masked or not) x (row-major or row-blocked q|k|v); long: S % 256 == 0 and the TAIL form
    assert len(spatial) == 4 and len(long_) == 2
    # attn_long_kernel runs two 512-thread workgroups per CU: 128 VGPRs per lane at most
    assert all(int(by[n][".vgpr_count"]) <= 128 for n in long_)


def test_asm_loads_waited_or_audited(audited_asm):
    srcs = _hip_sources()
    loads = {s: ck.asm_loads(open(s).read()) for s in srcs}
    form2 = {os.path.splitext(os.path.basename(s))[0] for s, l in loads.items() if any(f == "ii" for _, f in l)}
    assert ck.source_violations(srcs, audited_asm) == []  # every such source / header is audited
    assert form2 == {"attention", "attention_long_kernel"}
    # the LDS reads of both attention kernels are form (i): reads + wait in one statement
    common = ck.asm_loads(open(os.path.join(CSRC, "vp_common.h")).read())
    assert len(common) == 4 and all(f == "i" for _, f in common)  # base-address and immediate-offset forms


def _inject_after_first_asm_load(src_path, dst_path, make_line):
    lines = open(src_path).read().splitlines()
    for i, l in enumerate(lines):
        if l.strip().startswith("global_load_dwordx4") and lines[i - 1].strip() == ";;#ASMSTART":
            dst = l.split()[1].rstrip(",")
            first = int(re.match(r"v\[(\d+):", dst).group(1))
            lines.insert(i + 2, make_line(first))  # after ;;#ASMEND
            open(dst_path, "w").write("\n".join(lines) + "\n")
            return
    raise AssertionError("no asm load found")


@pytest.mark.parametrize("inject", ["\tv_mov_b32_e32 v250, v{r}",
                                    "\tscratch_store_dword off, v{r}, off ; 4-byte Folded Spill"])
def test_audit_rejects_access_in_flight(audited_asm, tmp_path, inject):
    src = [a for a in audited_asm if a.endswith("attention.s")][0]
    bad = tmp_path / "attention.s"
    _inject_after_first_asm_load(src, str(bad), lambda r: inject.format(r=r))
    v = ck.audit_asm(str(bad))
    assert v and "in flight" in v[0], v


def test_resource_check_rejects_scratch(tmp_path):
    if not os.path.exists(HIPCC):
        pytest.skip("hipcc not available")
    src = tmp_path / "spill.hip"
    src.write_text("""
#include <hip/hip_runtime.h>
__global__ void spill_kernel(float* o, const int* idx) {
  float a[96];
  for (int i = 0; i < 96; ++i) a[i] = o[i * 64 + threadIdx.x];
  o[threadIdx.x] = a[idx[threadIdx.x] % 96];
}
extern "C" void launch(float* o, const int* idx) { hipLaunchKernelGGL(spill_kernel, 1, 64, 0, 0, o, idx); }
""")
    lib = tmp_path / "libspill.so"
    subprocess.run([HIPCC, *FLAGS, "-fPIC", "-shared", str(src), "-o", str(lib)], check=True, capture_output=True)
    bad = ck.resource_violations(str(lib))
    assert bad and "private_segment_fixed_size" in bad[0], bad


def test_every_source_kernel_has_device_code(tmp_path):
    """`make` also refuses a library that lacks the device code of any __global__ function its sources
    define (a compile once dropped a whole translation unit's kernels silently, rc 0)."""
    lib = _native.library_path()
    srcs = _hip_sources()
    assert ck.missing_kernels(lib, srcs) == []
    extra = tmp_path / "extra.hip"
    extra.write_text("__global__ __launch_bounds__(64) void not_built_kernel(float* o) { o[0] = 1.f; }\n")
    assert ck.missing_kernels(lib, srcs + [str(extra)]) == ["not_built_kernel"]



@pytest.mark.parametrize("listing", ["attention.s"])
def test_audit_rejects_a_wait_count_too_high(audited_asm, tmp_path, listing):
    """vmcnt retires in issue order: the wait statement that retires the form-(ii) Q loads must leave
    at most the younger LDS-DMA pieces outstanding.  With its count raised by 4 the oldest Q loads are
    still in flight when the MFMAs read them, and the audit (which queues every vector-memory
    instruction in issue order) refuses the listing.  (attention_long.s is not a negative case: its
    chunk loop opens with a wait of its own that retires the Q loads before any MFMA reads them.)"""
    src = [a for a in audited_asm if a.endswith(listing)][0]
    assert ck.audit_asm(src) == []
    lines = open(src).read().splitlines()
    first_load = next(i for i, l in enumerate(lines)
                      if l.strip().startswith("global_load_dwordx4") and lines[i - 1].strip() == ";;#ASMSTART")
    k = next(i for i in range(first_load, len(lines)) if re.match(r"\s*s_waitcnt vmcnt\(\d+\)\s*$", lines[i])
             and lines[i - 1].strip() == ";;#ASMSTART")
    n = int(re.search(r"vmcnt\((\d+)\)", lines[k]).group(1))
    lines[k] = lines[k].replace(f"vmcnt({n})", f"vmcnt({n + 4})")
    bad = tmp_path / listing
    bad.write_text("\n".join(lines) + "\n")
    v = ck.audit_asm(str(bad))
    assert v and "in flight" in v[0], v
