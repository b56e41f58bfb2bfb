"""Build-time guards for the hand-written HIP kernels (run by `make`; tests/test_kernel_checks.py
runs the same checks on CPU).

  python tools/check_kernels.py resources LIB.so
      Every gfx950 kernel in LIB.so's offload bundle must have .private_segment_fixed_size 0 and
      .vgpr_spill_count 0 (read from the code object's AMDGPU metadata note).  A spill or a
      scratch slot means the register allocator ran out of room -- for the attention kernels
      whose asm loads the compiler does not track, that is the failure that faulted
      attn_long_pipe_kernel in round 3 (its asm Q-load destinations were spilled while the loads
      were still in flight).
  python tools/check_kernels.py sources SRC... [--asm FILE.s ...]
      Every inline-asm load with a VGPR destination in SRC must either carry its s_waitcnt in the
      same statement (cdna_hip_programming.md §5.7 item 1, form (i)) or, when it is retired by a
      later wait statement that names its destinations (form (ii)), its source file must be given
      as --asm assembly; the assembly is then audited: between such a load and the wait that
      retires it (in layout order) no compiler instruction and no other asm statement may read,
      write, copy or spill its destination registers.
  python tools/check_kernels.py report LIB.so
      VGPR / AGPR / scratch figures of every kernel (DESIGN.md quotes them).

Exit status 1 with a message naming the kernel / line on any violation."""

from __future__ import annotations

import os
import re
import struct
import sys

_MSGPACK = None


def _msgpack():
    global _MSGPACK
    if _MSGPACK is None:
        try:
            import msgpack
        except ImportError as e:  # the AMDGPU metadata note is a msgpack map
            raise SystemExit("check_kernels: the Python module 'msgpack' is required to read the kernels' "
                             "AMDGPU metadata (pip install msgpack); the library was not checked") from e
        _MSGPACK = msgpack
    return _MSGPACK


# ------------------------------------------------------------------------------------------------
# code object metadata
# ------------------------------------------------------------------------------------------------
def _elf_sections(data: bytes):
    if data[:4] != b"\x7fELF" or data[4] != 2:
        raise ValueError("not an ELF64 file")
    shoff, = struct.unpack_from("<Q", data, 0x28)
    shentsize, shnum, shstrndx = struct.unpack_from("<HHH", data, 0x3A)
    hdrs = []
    for i in range(shnum):
        name, typ, _flags, _addr, off, size = struct.unpack_from("<IIQQQQ", data, shoff + i * shentsize)
        hdrs.append((name, typ, off, size))
    stro = hdrs[shstrndx][2]
    out = {}
    for name, typ, off, size in hdrs:
        end = data.index(b"\0", stro + name)
        out[data[stro + name:end].decode()] = (typ, off, size)
    return out


def device_code_objects(lib_path: str, arch: str = "gfx950"):
    """The device code objects for `arch` in a hipcc-built shared library's .hip_fatbin bundle(s)."""
    data = open(lib_path, "rb").read()
    secs = _elf_sections(data)
    if ".hip_fatbin" not in secs:
        raise ValueError(f"{lib_path}: no .hip_fatbin section")
    _t, off, size = secs[".hip_fatbin"]
    fat = data[off:off + size]
    magic = b"__CLANG_OFFLOAD_BUNDLE__"
    cos = []
    pos = fat.find(magic)
    while pos >= 0:
        n, = struct.unpack_from("<Q", fat, pos + 24)
        p = pos + 32
        for _ in range(n):
            o, sz, tl = struct.unpack_from("<QQQ", fat, p)
            triple = fat[p + 24:p + 24 + tl].decode()
            p += 24 + tl
            if triple.endswith(arch) and sz > 0:
                cos.append(fat[pos + o:pos + o + sz])
        pos = fat.find(magic, pos + 1)
    if not cos:
        raise ValueError(f"{lib_path}: no {arch} code object in the offload bundle")
    return cos


def kernel_metadata(code_object: bytes):
    """amdhsa.kernels of the NT_AMDGPU_METADATA note (msgpack)."""
    secs = _elf_sections(code_object)
    for name, (typ, off, size) in secs.items():
        if typ != 7:  # SHT_NOTE
            continue
        p, end = off, off + size
        while p + 12 <= end:
            namesz, descsz, ntype = struct.unpack_from("<III", code_object, p)
            nm = code_object[p + 12:p + 12 + namesz].rstrip(b"\0")
            dpos = p + 12 + ((namesz + 3) & ~3)
            desc = code_object[dpos:dpos + descsz]
            p = dpos + ((descsz + 3) & ~3)
            if nm == b"AMDGPU" and ntype == 32:
                return _msgpack().unpackb(desc, raw=False)["amdhsa.kernels"]
    raise ValueError("no AMDGPU metadata note")


def kernels(lib_path: str):
    out = []
    for co in device_code_objects(lib_path):
        out.extend(kernel_metadata(co))
    return out


def resource_violations(lib_path: str):
    bad = []
    for k in kernels(lib_path):
        name = k[".name"]
        # (SGPR spills land in VGPR lanes via v_writelane -- no memory, no scratch -- and are
        # reported by `report`, not refused)
        for key in (".private_segment_fixed_size", ".vgpr_spill_count"):
            if int(k.get(key, 0)) != 0:
                bad.append(f"{name}: {key} = {k[key]}")
    return bad


_GLOBAL_FN = re.compile(r"__global__\s+(?:__launch_bounds__\s*\([^)]*\)\s*)?void\s+(\w+)\s*\(")


def missing_kernels(lib_path: str, sources):
    """__global__ functions defined in `sources` of which the library holds no device code at all --
    the failure of a host + device compile that silently dropped a translation unit's kernels (seen
    once with a non-literal cache-policy argument to an LDS-DMA builtin: object built, rc 0, kernels
    and their stubs gone, the library still linked)."""
    have = set()
    for k in kernels(lib_path):
        m = re.match(r"_ZN2vp12_GLOBAL__N_1\d+(\w+?)(?:I|E|v|P)", k[".name"])
        have.add(m.group(1) if m else k[".name"])
    want = set()
    for src in sources:
        if src.endswith((".hip", ".h")) and os.path.exists(src):
            want.update(_GLOBAL_FN.findall(open(src).read()))
    names = " ".join(k[".name"] for k in kernels(lib_path))
    return sorted(w for w in want if w not in have and w not in names)


# ------------------------------------------------------------------------------------------------
# inline-asm loads in the sources
# ------------------------------------------------------------------------------------------------
_LOAD_MN = re.compile(r"\b(global_load|buffer_load|flat_load|scratch_load|ds_read|ds_load)\w*")
_ASM_STMT = re.compile(r"asm\s+volatile\s*\((.*?)\)\s*;", re.S)


def _split_outside_strings(body: str, sep: str):
    """`body` split at `sep` characters that are not inside a "..." literal (asm text such as
    "ds_read_b64_tr_b16 %1, %8 offset:1024" holds colons of its own)."""
    parts, cur, in_str, esc = [], [], False, False
    for ch in body:
        if in_str:
            cur.append(ch)
            if esc:
                esc = False
            elif ch == "\\":
                esc = True
            elif ch == '"':
                in_str = False
            continue
        if ch == '"':
            in_str = True
            cur.append(ch)
        elif ch == sep:
            parts.append("".join(cur))
            cur = []
        else:
            cur.append(ch)
    parts.append("".join(cur))
    return parts


def asm_loads(src: str):
    """(line, form) of every asm statement in `src` that loads into a VGPR output; form 'i' when
    the statement also waits (s_waitcnt) for them, else 'ii'."""
    out = []
    for m in _ASM_STMT.finditer(src):
        body = m.group(1)
        parts = _split_outside_strings(body, ":")
        text = parts[0]
        outputs = parts[1] if len(parts) > 1 else ""
        if not _LOAD_MN.search(text) or " lds" in text or "_lds" in text:
            continue
        if not re.search(r'"=&?v"', outputs):
            continue
        line = src.count("\n", 0, m.start()) + 1
        out.append((line, "i" if "s_waitcnt" in text else "ii"))
    return out


_REG1 = re.compile(r"\bv(\d+)\b")
_REGN = re.compile(r"\bv\[(\d+):(\d+)\]")


def _regs(operands: str):
    s = set()
    for a, b in _REGN.findall(operands):
        s.update(range(int(a), int(b) + 1))
    for a in _REG1.findall(_REGN.sub(" ", operands)):
        s.add(int(a))
    return s


def _kind(mn: str):
    return "lgkm" if mn.startswith("ds_") else "vm"


_VMEM_MN = re.compile(r"^(global|buffer|flat|scratch)_(load|store|atomic)\w*")
_WAIT_CNT = re.compile(r"(vmcnt|lgkmcnt)\((\d+)\)")


def audit_asm(path: str):
    """Walk a hipcc -S listing in layout order and report any access to the destination registers
    of a form-(ii) asm load between the load and the wait that retires it.

    vmcnt retires in issue order: every vector-memory instruction (loads, stores, LDS-DMA pieces;
    the compiler's and asm statements' alike) is queued as it is issued, and an `s_waitcnt vmcnt(N)`
    retires all but the N youngest -- an asm load is retired only when it is older than those N, so
    a wait count too high for the loads it must cover is caught (their registers are then read while
    still in flight).  lgkm loads are retired by any lgkmcnt wait in an asm statement and by a
    compiler lgkmcnt(0) (the product's asm LDS reads wait in their own statement, form (i))."""
    lines = open(path).read().splitlines()
    bad = []
    pending = {}  # reg -> (kind, line of the load)
    vmq = []      # vector-memory operations in issue order: the destination regs of asm loads, or None
    in_asm, block, block_start, func = False, [], 0, "?"

    def retire_lgkm():
        for r in [r for r, (k, _) in pending.items() if k == "lgkm"]:
            del pending[r]

    def wait_vm(n):
        nonlocal vmq
        old, vmq = (vmq, []) if n == 0 else (vmq[:-n], vmq[-n:])
        for regs in old:
            for r in regs or ():
                if r in pending and pending[r][0] == "vm":
                    del pending[r]

    def waits_in(text):
        for kind, n in _WAIT_CNT.findall(text):
            if kind == "vmcnt":
                wait_vm(int(n))
            elif kind == "lgkmcnt":
                yield int(n)

    for no, raw in enumerate(lines, 1):
        ln = raw.split(";")[0].strip() if not raw.strip().startswith(";;#ASM") else raw.strip()
        if raw.strip() == ";;#ASMSTART":
            in_asm, block, block_start = True, [], no
            continue
        if raw.strip() == ";;#ASMEND":
            in_asm = False
            insts = [b for b in block if b and not b.startswith(";")]
            loads = [b for b in insts if _LOAD_MN.match(b.split()[0]) and "lds" not in b.split()[0]
                     and not b.split()[0].endswith("_lds")]
            touched = set()
            for b in insts:
                mn, _, ops = b.partition(" ")
                if mn == "s_waitcnt":
                    continue
                if b in loads:
                    dst, _, rest = ops.partition(",")
                    touched |= _regs(rest)
                else:
                    touched |= _regs(ops)
            hit = touched & set(pending)
            if hit:
                bad.append(f"{path}:{block_start} ({func}): asm statement reads v{sorted(hit)} while the "
                           f"load at line {pending[min(hit)][1]} is in flight")
            for b in insts:
                mn, _, ops = b.partition(" ")
                if mn == "s_waitcnt":
                    if list(waits_in(ops)):
                        retire_lgkm()
                    continue
                if b in loads:
                    regs = _regs(ops.partition(",")[0])
                    for r in regs:
                        pending[r] = (_kind(mn), no)
                    if _kind(mn) == "vm":
                        vmq.append(regs)
                elif _VMEM_MN.match(mn):
                    vmq.append(None)
            continue
        if in_asm:
            block.append(raw.strip())
            continue
        if not ln or ln.startswith(".") or ln.endswith(":"):
            if ln.startswith(".Lfunc_end") or ln.startswith(".amdhsa_kernel") or (
                    ln.endswith(":") and not ln.startswith(".")):
                if pending and ln.startswith(".Lfunc_end"):
                    bad.append(f"{path}:{no} ({func}): function ends with asm loads never retired "
                               f"(lines {sorted({v[1] for v in pending.values()})})")
                pending.clear()
                vmq = []
                if ln.endswith(":") and not ln.startswith("."):
                    func = ln[:-1]
            continue
        mn, _, ops = ln.partition(" ")
        if mn == "s_waitcnt":
            if 0 in list(waits_in(ops)):
                retire_lgkm()
            continue
        hit = _regs(ops) & set(pending)
        if hit:
            bad.append(f"{path}:{no} ({func}): compiler instruction '{ln}' touches v{sorted(hit)} while the "
                       f"asm load at line {pending[min(hit)][1]} is in flight")
        if _VMEM_MN.match(mn):
            vmq.append(None)
            if len(vmq) > 256 and not any(vmq[:-64]):
                vmq = vmq[-64:]  # vmcnt counts at most 63
    return bad


def source_violations(srcs, asm_files):
    """A source with form-(ii) asm loads must have an audited listing; a header's, a listing of a
    source among `srcs` that includes it."""
    bad = []
    audited = {os.path.splitext(os.path.basename(a))[0] for a in asm_files}
    texts = {s: open(s).read() for s in srcs}
    for s in srcs:
        loads = asm_loads(texts[s])
        if any(f == "ii" for _, f in loads):
            stem = os.path.splitext(os.path.basename(s))[0]
            if s.endswith(".h"):
                inc = f'#include "{os.path.basename(s)}"'
                users = {os.path.splitext(os.path.basename(t))[0] for t, txt in texts.items() if inc in txt}
                if users & audited:
                    continue
            if stem not in audited:
                bad.append(f"{s}: asm loads retired by a later wait (lines "
                           f"{[l for l, f in loads if f == 'ii']}) need an --asm audit of this file")
    for a in asm_files:
        bad.extend(audit_asm(a))
    return bad


def main(argv):
    if len(argv) < 2:
        print(__doc__)
        return 2
    cmd = argv[1]
    if cmd == "resources":
        bad = resource_violations(argv[2])
        missing = missing_kernels(argv[2], argv[3:])
        if missing:
            print("check_kernels: no device code for kernels defined in the sources:\n  " + "\n  ".join(missing),
                  file=sys.stderr)
            return 1
        n = len(kernels(argv[2]))
        if bad:
            print("check_kernels: scratch / spills in product kernels:\n  " + "\n  ".join(bad), file=sys.stderr)
            return 1
        print(f"check_kernels: {n} kernels in {os.path.basename(argv[2])}: no scratch, no spills")
        return 0
    if cmd == "sources":
        args = argv[2:]
        srcs = [a for a in args if not a.endswith(".s") and a != "--asm"]
        asm = [a for a in args if a.endswith(".s")]
        bad = source_violations(srcs, asm)
        if bad:
            print("check_kernels: unsafe asm loads:\n  " + "\n  ".join(bad), file=sys.stderr)
            return 1
        n = sum(len(asm_loads(open(s).read())) for s in srcs)
        print(f"check_kernels: {n} asm VGPR loads in {len(srcs)} sources, {len(asm)} listings audited: ok")
        return 0
    if cmd == "report":
        for k in sorted(kernels(argv[2]), key=lambda k: k[".name"]):
            print(f"{k['.name']}: vgpr {k.get('.vgpr_count')} agpr {k.get('.agpr_count')} "
                  f"sgpr {k.get('.sgpr_count')} (spilled to VGPR lanes {k.get('.sgpr_spill_count')}) "
                  f"scratch {k.get('.private_segment_fixed_size')} vgpr-spills {k.get('.vgpr_spill_count')} "
                  f"lds {k.get('.group_segment_fixed_size')}")
        return 0
    print(__doc__)
    return 2


if __name__ == "__main__":
    sys.exit(main(sys.argv))
