"""Code-object metadata of libhyres_hip.so's gfx950 kernels (register allocation, LDS, block size) and the
co-residency "holes" they leave: the VGPRs of a SIMD that one kernel's resident waves do not claim, in which waves of
ANOTHER kernel (another stream) can run beside them. DESIGN §4 "Cross-kernel interference" is why that matters.

    python scripts/kernel_meta.py [path/to/libhyres_hip.so] [--all]

Reads the .hip_fatbin section with llvm-objcopy, unbundles the gfx950 code object with clang-offload-bundler and
parses the AMDGPU metadata note (llvm-readelf --notes). Host tools only: no GPU.
"""
from __future__ import annotations

import os
import re
import subprocess
import sys
import tempfile

import yaml

LLVM = "/opt/rocm/lib/llvm/bin"
VGPRS_PER_SIMD = 512
LDS_PER_CU = 163840
GRANULE = 8


def _tool(name: str) -> str:
    return os.path.join(LLVM, name)


def available() -> bool:
    return all(os.path.exists(_tool(t)) for t in ("llvm-objcopy", "clang-offload-bundler", "llvm-readelf",
                                                   "llvm-objdump"))


def _code_objects(so_path: str, td: str, arch: str) -> list[str]:
    """Unbundle the gfx950 code object of every translation unit in the library's .hip_fatbin into ``td``."""
    magic = b"__CLANG_OFFLOAD_BUNDLE__"
    fat = os.path.join(td, "fat")
    subprocess.run([_tool("llvm-objcopy"), f"--dump-section=.hip_fatbin={fat}", so_path, os.path.join(td, "x")],
                   check=True, capture_output=True)
    blob = open(fat, "rb").read()
    starts = [m.start() for m in re.finditer(re.escape(magic), blob)]  # one bundle per translation unit
    cos = []
    for i, s0 in enumerate(starts):
        part, co = os.path.join(td, f"b{i}"), os.path.join(td, f"co{i}")
        with open(part, "wb") as f:
            f.write(blob[s0:starts[i + 1] if i + 1 < len(starts) else len(blob)])
        subprocess.run([_tool("clang-offload-bundler"), "--unbundle", "--type=o", f"--input={part}",
                        f"--targets=hipv4-amdgcn-amd-amdhsa--{arch}", f"--output={co}"], check=True,
                       capture_output=True)
        cos.append(co)
    return cos


def disassembly(so_path: str, arch: str = "gfx950") -> dict[str, list[str]]:
    """{mangled kernel name: its instructions (one string each, comments stripped)} from llvm-objdump."""
    out: dict[str, list[str]] = {}
    with tempfile.TemporaryDirectory() as td:
        for co in _code_objects(so_path, td, arch):
            txt = subprocess.run([_tool("llvm-objdump"), "-d", "--no-show-raw-insn", co], check=True,
                                 capture_output=True, text=True).stdout
            cur = None
            for line in txt.splitlines():
                m = re.match(r"^[0-9a-f]+ <(.*)>:$", line)
                if m:
                    cur = out.setdefault(m.group(1), [])
                    continue
                ins = line.split("//")[0].strip()
                if cur is not None and ins and not ins.endswith(":"):
                    cur.append(ins)
    return out


_REG = re.compile(r"(?<![\w])([va])(?:\[(\d+):(\d+)\]|(\d+)(?!\w))")


def _regs(text: str) -> set:
    out = set()
    for m in _REG.finditer(text):
        if m.group(4) is not None:
            out.add((m.group(1), int(m.group(4))))
        else:
            out.update((m.group(1), r) for r in range(int(m.group(2)), int(m.group(3)) + 1))
    return out


def lds_read_hazards(instrs: list[str]) -> list[tuple[str, str]]:
    """Instructions that touch (read or overwrite) the destination VGPRs of an LDS read that has not been waited for.

    Linear scan in program order: every LGKM operation (ds_*, s_load*, s_buffer_load*, s_sendmsg) joins an in-order
    queue; ``s_waitcnt lgkmcnt(N)`` retires all but the N most recent; an instruction whose operands overlap the
    destination of a still-queued ds_read is a hazard. This is the check a hand-issued ``ds_read_b128`` (inline asm,
    waited for by a hand-counted ``s_waitcnt``, conv.hip conv3x3_wres_bf6_kernel V & 1) needs: the compiler treats an
    asm output as ready at once and could place a copy of it before the wait. Compiler-issued reads pass by
    construction, which makes the scan of every kernel its own calibration."""
    q: list[tuple[str, set]] = []
    bad = []
    for ins in instrs:
        op = ins.split()[0]
        if op.startswith("s_waitcnt"):
            m = re.search(r"lgkmcnt\((\d+)\)", ins)
            if m:
                n = int(m.group(1))
                del q[:max(0, len(q) - n)]
            continue
        operands = ins[len(op):]
        rs = _regs(operands)
        for src, dst in q:
            if dst & rs:
                bad.append((src, ins))
        if op.startswith(("ds_read", "ds_load")):
            q.append((ins, _regs(operands.split(",")[0])))
        elif op.startswith(("ds_", "s_load", "s_buffer_load", "s_sendmsg")):
            q.append((ins, set()))
    return bad


def kernels(so_path: str, arch: str = "gfx950") -> list[dict]:
    """One dict per kernel: name, vgpr, agpr, accum_offset-free allocation, lds, threads, sgpr, scratch."""
    docs = []
    with tempfile.TemporaryDirectory() as td:
        for co in _code_objects(so_path, td, arch):
            notes = subprocess.run([_tool("llvm-readelf"), "--notes", co], check=True, capture_output=True,
                                   text=True).stdout
            m = re.search(r"^\s*---\n(.*?)^\s*\.\.\.\s*$", notes, re.S | re.M)
            docs.append(yaml.safe_load(m.group(1)))
    out = []
    for k in (k for d in docs for k in d["amdhsa.kernels"]):
        vg, ag = int(k[".vgpr_count"]), int(k.get(".agpr_count", 0))
        # gfx90a+: .vgpr_count is already the unified total (the arch VGPRs aligned to 4, then the AGPRs at
        # accum_offset; LLVM's NumVGPRsForWavesPerEU) — 395 on a kernel cannot be arch registers alone (v0..v255).
        # The allocation granule is 8
        total = vg
        alloc = max(GRANULE, -(-total // GRANULE) * GRANULE)
        out.append({"name": k[".name"], "vgpr": vg, "agpr": ag, "alloc": alloc,
                    "lds": int(k[".group_segment_fixed_size"]), "threads": int(k[".max_flat_workgroup_size"]),
                    "sgpr": int(k[".sgpr_count"]), "scratch": int(k[".private_segment_fixed_size"])})
    return out


def residency(k: dict) -> dict:
    """How one kernel occupies a CU when it fills the chip alone: blocks per CU (LDS, VGPR and wave limits), waves
    per SIMD, and the VGPRs per SIMD its waves leave free (the hole another kernel's waves can take)."""
    waves_per_block = -(-k["threads"] // 64)
    per_simd_per_block = -(-waves_per_block // 4)
    by_vgpr = (VGPRS_PER_SIMD // k["alloc"]) // per_simd_per_block
    by_lds = LDS_PER_CU // k["lds"] if k["lds"] else 1 << 30
    by_waves = 32 // waves_per_block
    blocks = max(0, min(by_vgpr, by_lds, by_waves))
    wps = blocks * per_simd_per_block
    hole = VGPRS_PER_SIMD - wps * k["alloc"]
    lds_left = LDS_PER_CU - blocks * k["lds"]
    return {"blocks_per_cu": blocks, "waves_per_simd": wps, "hole_vgprs": hole, "lds_left": lds_left,
            "lds_limited": by_lds <= min(by_vgpr, by_waves)}


def demangle(names: list[str]) -> list[str]:
    try:
        r = subprocess.run(["c++filt"], input="\n".join(names), capture_output=True, text=True, check=True)
        return r.stdout.splitlines()
    except Exception:  # noqa: BLE001 - c++filt absent: mangled names
        return names


def main(argv: list[str]) -> None:
    here = os.path.dirname(os.path.abspath(__file__))
    so = next((a for a in argv if a.endswith(".so")), os.path.join(
        os.path.dirname(here), "hyres-residual-enhanced-hybrid-image-compression_amd", "hyres_hip", "libhyres_hip.so"))
    ks = kernels(so)
    names = demangle([k["name"] for k in ks])
    print(f"{'kernel':70s} {'thr':>4s} {'vgpr':>4s} {'agpr':>4s} {'alloc':>5s} {'LDS':>7s} {'blk/CU':>6s} "
          f"{'w/SIMD':>6s} {'hole':>5s}")
    for k, n in sorted(zip(ks, names), key=lambda t: t[1]):
        r = residency(k)
        if "--all" not in argv and not (r["lds_limited"] and r["hole_vgprs"] > 0):
            continue
        print(f"{n[:70]:70s} {k['threads']:4d} {k['vgpr']:4d} {k['agpr']:4d} {k['alloc']:5d} {k['lds']:7d} "
              f"{r['blocks_per_cu']:6d} {r['waves_per_simd']:6d} {r['hole_vgprs']:5d}")


if __name__ == "__main__":
    main(sys.argv[1:])
