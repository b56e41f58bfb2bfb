"""Summarise rocprofv3 --pmc CSVs (tools/pmc_passes.sh) per kernel: mean per dispatch,
plus derived clock / MFMA-busy / HBM-byte figures (MI355X_MICROARCH.md rules:
GRBM_GUI_ACTIVE is summed over 8 XCDs; FETCH_SIZE reads 1/2 of wide streaming reads)."""
import csv
import glob
import os
import re
import sys
from collections import defaultdict


def short(name):
    m = re.search(r"(\w+_kernel\w*)<([^>]*)>", name)
    if "Cijk" in name:
        return "hipblaslt:" + name.split("_")[-2]
    if m:
        return f"{m.group(1)}<{m.group(2)}>"
    return name.split("(")[0][-60:]


root = sys.argv[1]
vals = defaultdict(lambda: defaultdict(list))
dur = defaultdict(list)
for f in glob.glob(os.path.join(root, "p*", "**", "*counter_collection.csv"), recursive=True):
    for r in csv.DictReader(open(f)):
        k = short(r["Kernel_Name"])
        vals[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
        dur[k].append((float(r["End_Timestamp"]) - float(r["Start_Timestamp"])) * 1e-9)
for k, cs in vals.items():
    if not (k.startswith("gemm") or k.startswith("hipblas") or "attn" in k or "layernorm" in k or "ln_" in k):
        continue
    m = {c: sum(v) / len(v) for c, v in cs.items()}
    t = sum(dur[k]) / len(dur[k])
    print(f"{k}  avg dispatch {t*1e6:.1f} us")
    for c, v in sorted(m.items()):
        print(f"   {c:28s} {v:16.4g}")
    if "GRBM_GUI_ACTIVE" in m:
        clk = m["GRBM_GUI_ACTIVE"] / 8 / t
        print(f"   => effective clock {clk/1e9:.2f} GHz")
        if "SQ_VALU_MFMA_BUSY_CYCLES" in m:
            busy = m["SQ_VALU_MFMA_BUSY_CYCLES"] / (m["GRBM_GUI_ACTIVE"] / 8 * 256 * 4)
            print(f"   => MFMA busy fraction (per SIMD) {busy:.3f}")
    if "FETCH_SIZE" in m:
        print(f"   => HBM read ~ {2*m['FETCH_SIZE']*1024/1e6:.1f} MB (FETCH_SIZE x2, gfx950 rule)")
    if "WRITE_SIZE" in m:
        print(f"   => HBM write ~ {m['WRITE_SIZE']*1024/1e6:.1f} MB")


# --json OUT WORKLOAD: per-launch HBM bytes of every kernel symbol seen in the FETCH_SIZE and
# WRITE_SIZE passes, keyed by the short symbol (e.g. "gemm_bf16_w4_kernel<9, 512, 0>"), with the
# source fingerprint of the build that ran (bench.py quotes a record only for the same sources,
# workload and symbol): 2 x FETCH_SIZE (gfx950 rule) + WRITE_SIZE, KiB counters.
if len(sys.argv) > 4 and sys.argv[2] == "--json":
    import json
    sys.path[:0] = [os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                 "videoprism-mlx_amd")]
    from videoprism import _native
    out = {"source": f"rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE in separate passes over "
                     f"`bench.py --workload {sys.argv[4].removesuffix('_f32')}"
                     f"{' --dtype f32' if sys.argv[4].endswith('_f32') else ''}` (tools/pmc_traffic.sh); hbm_bytes_per_launch "
                     "= 2*FETCH_SIZE*1024 + WRITE_SIZE*1024 (MI355X_MICROARCH.md HBM section: FETCH_SIZE "
                     "reads half of wide streaming reads on gfx950; Infinity-Cache hits are counted)",
           "workload": sys.argv[4], "src_hash": _native.source_fingerprint(), "kernels": {}}
    for k, cs in vals.items():
        if "FETCH_SIZE" not in cs or "WRITE_SIZE" not in cs:
            continue
        f = sum(cs["FETCH_SIZE"]) / len(cs["FETCH_SIZE"])
        w = sum(cs["WRITE_SIZE"]) / len(cs["WRITE_SIZE"])
        out["kernels"][k] = {"fetch_bytes": 2 * f * 1024, "write_bytes": w * 1024,
                             "hbm_bytes_per_launch": 2 * f * 1024 + w * 1024,
                             "dispatches": len(cs["FETCH_SIZE"])}
    with open(sys.argv[3], "w") as fo:
        json.dump(out, fo, indent=1)
    print("wrote", sys.argv[3])
