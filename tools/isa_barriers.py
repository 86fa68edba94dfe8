#!/usr/bin/env python3
"""Static barrier check of the shipped gfx950 ISA (CPU only: disassembles
the code objects inside a built .so, runs no GPU code).

A workgroup barrier (s_barrier) hangs the workgroup when its waves do not
all reach it the same number of times.  Two ways code generation can break
that for a kernel whose source keeps every barrier on workgroup-uniform
control flow, and what this tool checks for each:

1. a barrier inside an EXEC-masked (lane-divergent) region: a wave whose
   lanes are all inactive jumps over the region (s_cbranch_execz), or leaves
   a divergent loop on a different trip than its neighbours (s_cbranch_execnz
   back edge).  Check: no s_barrier between a forward execz/execnz branch and
   its target, nor inside the body of a loop closed by an exec branch;
2. a loop iteration whose paths differ in their barrier count.

One check covers both: the BARRIER FRONTIER of a point is the set of
barriers a wave can reach next from it (a fixpoint over the CFG, loops
included).  At every branch on EXEC (s_cbranch_execz / execnz: the lanes of
the wave decide it, so waves may go different ways), both directions must
reach the same next barriers -- the divergent region reconverges before any
barrier.  A direction whose only continuation is the program end is
compatible with any (a wave that has ended no longer counts at a barrier).
Scalar branches (SCC / VCC) are wave-uniform by construction; whether their
condition is also WORKGROUP-uniform is the source's contract (every such
condition in these kernels derives from blockIdx, kernel arguments or LDS
values read after a barrier), so per loop the tool reports the barriers
per iteration (min and max over the paths of one trip) for review.

Plus the waitcnt census the round-2 hang note asked for: per loop, the
number of s_barrier, s_waitcnt vmcnt / lgkmcnt, buffer_load ... lds and
MFMA instructions.

    python tools/isa_barriers.py grid_amd/_lib/libgridhip.so [--kernels k_gram8,k_phase2] [--json]
"""
from __future__ import annotations

import argparse
import json
import re
import struct
import subprocess
import sys
import tempfile
from pathlib import Path

LLVM = "/opt/rocm/lib/llvm/bin"
MAGIC = b"__CLANG_OFFLOAD_BUNDLE__"
BRANCH_RE = re.compile(r"^s_(c?branch)(_\w+)?\b")
ADDR_RE = re.compile(r"//\s*([0-9A-Fa-f]{8,16}):")
TGT_RE = re.compile(r"<([^>+]+)\+0x([0-9a-fA-F]+)>\s*$")
EXEC_WRITE = re.compile(r"^s_\w*saveexec\w*\s|^s_\w+\s+exec\s*,")


def code_objects(so: str) -> list[bytes]:
    """The gfx950 code objects of a HIP shared library (.hip_fatbin bundles)."""
    with tempfile.TemporaryDirectory() as td:
        fb = Path(td) / "fatbin.bin"
        subprocess.run([f"{LLVM}/llvm-objcopy", f"--dump-section=.hip_fatbin={fb}", so, f"{td}/x.so"],
                       check=True, capture_output=True)
        d = fb.read_bytes()
    out = []
    for m in re.finditer(re.escape(MAGIC), d):
        s = m.start()
        n = struct.unpack_from("<Q", d, s + 24)[0]
        p = s + 32
        for _ in range(n):
            off, size, tl = struct.unpack_from("<QQQ", d, p)
            p += 24
            triple = d[p:p + tl].decode()
            p += tl
            if "gfx950" in triple:
                out.append(d[s + off:s + off + size])
    return out


def disassemble(elf: bytes) -> str:
    with tempfile.NamedTemporaryFile(suffix=".elf") as f:
        f.write(elf)
        f.flush()
        r = subprocess.run([f"{LLVM}/llvm-objdump", "-d", "--no-show-raw-insn", f.name], check=True,
                           capture_output=True, text=True)
    return r.stdout


def demangle(names):
    r = subprocess.run(["c++filt"], input="\n".join(names), capture_output=True, text=True,
                       check=True)
    return r.stdout.splitlines()


def short_name(dem: str) -> str:
    """'void k_gram8<0, true, 1, 3>(unsigned short const*, ...)' -> 'k_gram8<0, true, 1, 3>'."""
    s = dem[5:] if dem.startswith("void ") else dem
    s = s.replace("(anonymous namespace)::", "")
    depth = 0
    for i, ch in enumerate(s):
        if ch == "<":
            depth += 1
        elif ch == ">":
            depth -= 1
        elif ch == "(" and depth == 0:
            return s[:i]
    return s


class Insn:
    __slots__ = ("addr", "op", "text", "target")

    def __init__(self, addr, op, text, target):
        self.addr, self.op, self.text, self.target = addr, op, text, target


def parse_functions(dis: str) -> dict[str, list[Insn]]:
    """{demangled name: instructions} from llvm-objdump -d output."""
    funcs, cur, name, base = {}, None, None, 0
    for line in dis.splitlines():
        m = re.match(r"^([0-9a-fA-F]+) <(.+)>:$", line)
        if m:
            name, base = m.group(2), int(m.group(1), 16)
            cur = funcs.setdefault(name, [])
            continue
        if cur is None or not line.startswith("\t"):
            continue
        body = line.strip()
        am = ADDR_RE.search(body)
        if not am:
            continue
        addr = int(am.group(1), 16)
        text = body[: am.start()].strip()
        op = text.split()[0] if text else ""
        tgt = None
        tm = TGT_RE.search(body)
        if tm and op.startswith("s_") and "branch" in op:
            tgt = base + int(tm.group(2), 16) if tm.group(1) == name else None
        cur.append(Insn(addr, op, text, tgt))
    return funcs


def is_branch(op):
    return op == "s_branch" or op.startswith("s_cbranch_")


def analyse(insns: list[Insn]) -> dict:
    """The barrier-frontier check of one function and its per-loop census
    (see the module docstring)."""
    if not insns:
        return {"barriers": 0, "errors": [], "loops": []}
    idx = {ins.addr: i for i, ins in enumerate(insns)}
    errors = []
    # ---- basic blocks and edges ----
    leaders = {0}
    for i, ins in enumerate(insns):
        if is_branch(ins.op) or ins.op in ("s_endpgm", "s_barrier"):
            if i + 1 < len(insns):
                leaders.add(i + 1)          # a barrier ends its block: frontiers are per barrier
            if ins.target is not None and ins.target in idx:
                leaders.add(idx[ins.target])
        if is_branch(ins.op) and ins.target is None:
            errors.append(f"{ins.addr:x}: {ins.op} to an address outside the function")
    starts = sorted(leaders)
    blk_of, blocks = {}, []
    for k, st in enumerate(starts):
        e = starts[k + 1] if k + 1 < len(starts) else len(insns)
        blocks.append((st, e))
        for i in range(st, e):
            blk_of[i] = k
    succ = []
    for k, (st, e) in enumerate(blocks):
        last = insns[e - 1]
        out = []
        if last.op == "s_endpgm":
            pass
        elif last.op == "s_branch":
            if last.target in idx:
                out.append(blk_of[idx[last.target]])
        else:
            if last.op.startswith("s_cbranch_") and last.target in idx:
                out.append(blk_of[idx[last.target]])
            if k + 1 < len(blocks):
                out.append(k + 1)
        succ.append(out)
    first_bar = []
    for st, e in blocks:
        fb = next((i for i in range(st, e) if insns[i].op == "s_barrier"), None)
        first_bar.append(fb)
    # ---- barrier frontier: the barriers (or END) a wave can reach next from
    # the start of each block; fixpoint over the CFG (loops included) ----
    front = [set() for _ in blocks]
    changed = True
    while changed:
        changed = False
        for k in range(len(blocks) - 1, -1, -1):
            if first_bar[k] is not None:
                f = {insns[first_bar[k]].addr}
            else:
                f = set()
                if insns[blocks[k][1] - 1].op == "s_endpgm":
                    f.add("END")
                for s2 in succ[k]:
                    f |= front[s2]
            if f != front[k]:
                front[k] = f
                changed = True
    # ---- the check: every EXEC-dependent branch reconverges before a barrier ----
    for k, (st, e) in enumerate(blocks):
        last = insns[e - 1]
        if last.op not in ("s_cbranch_execz", "s_cbranch_execnz") or len(succ[k]) != 2:
            continue
        # only a branch right after the block narrowed EXEC splits the wave's
        # lanes from its neighbours' (an if: s_and_saveexec; a loop exit:
        # s_andn2 exec); without an EXEC write in the block the branch is a
        # skip guard taken only when EXEC was already empty on entry, i.e.
        # inside a region some enclosing divergent branch already covers
        if not any(EXEC_WRITE.match(insns[i].text) for i in range(st, e - 1)):
            continue
        # a wave that ends (s_endpgm) no longer takes part in barriers, so a
        # direction whose only continuation is the end is compatible with any
        fa, fb = front[succ[k][0]] - {"END"}, front[succ[k][1]] - {"END"}
        if fa and fb and fa != fb:
            fmt = lambda f: "{" + ", ".join(sorted(f"{x:x}" for x in f)) + "}"
            errors.append(f"{last.addr:x}: {last.op}: the two directions reach different next barriers "
                          f"{fmt(fa)} vs {fmt(fb)}")
    # ---- census per loop (back edge k -> h): barriers per iteration (min, max
    # over paths through the iteration; inner loops counted once), waits, DMA ----
    nbar = [sum(1 for i in range(st, e) if insns[i].op == "s_barrier") for st, e in blocks]
    loops = []
    for k, out in enumerate(succ):
        for h in out:
            if h > k:
                continue
            lo, hi = {h: nbar[h]}, {h: nbar[h]}
            for b in range(h, k + 1):
                if b not in lo:
                    continue
                for s2 in succ[b]:
                    if b < s2 <= k:
                        lo[s2] = min(lo.get(s2, lo[b] + nbar[s2]), lo[b] + nbar[s2])
                        hi[s2] = max(hi.get(s2, hi[b] + nbar[s2]), hi[b] + nbar[s2])
            cnt = {"s_barrier": 0, "vmcnt": 0, "lgkmcnt": 0, "lds_dma": 0, "mfma": 0, "scratch": 0}
            for i in range(blocks[h][0], blocks[k][1]):
                t, op = insns[i].text, insns[i].op
                if op == "s_barrier":
                    cnt["s_barrier"] += 1
                elif op == "s_waitcnt":
                    cnt["vmcnt"] += "vmcnt" in t and "vmcnt(63)" not in t
                    cnt["lgkmcnt"] += "lgkmcnt" in t and "lgkmcnt(15)" not in t
                elif op.startswith("buffer_load") and t.rstrip().endswith(" lds"):
                    cnt["lds_dma"] += 1
                elif op.startswith("v_mfma"):
                    cnt["mfma"] += 1
                elif op.startswith("scratch_"):
                    cnt["scratch"] += 1          # a spill reload's vmcnt wait would drain an LDS-DMA ring
            loops.append({"head": f"{insns[blocks[h][0]].addr:x}", "end": f"{insns[blocks[k][1] - 1].addr:x}",
                          "insns": blocks[k][1] - blocks[h][0],
                          "back_edge": insns[blocks[k][1] - 1].op,
                          "barriers_per_iter": [lo.get(k), hi.get(k)], **cnt})
    for lp in loops:                      # innermost: no other loop nested inside its range
        h0, e0 = int(lp["head"], 16), int(lp["end"], 16)
        lp["innermost"] = not any(h0 <= int(o["head"], 16) and int(o["end"], 16) <= e0 and
                                  (o["head"], o["end"]) != (lp["head"], lp["end"]) for o in loops)
    return {"barriers": sum(nbar), "errors": errors, "loops": loops}


def check(funcs: dict[str, list[Insn]], pattern: str) -> dict:
    pats = [p for p in pattern.split(",") if p]
    res = {}
    names = list(funcs)
    for name, dem in zip(names, demangle(names)):
        insns = funcs[name]
        short = short_name(dem)
        if pats and not any(p in short for p in pats):
            continue
        if not any(ins.op == "s_barrier" for ins in insns):
            continue
        res[short] = analyse(insns)
    return res


def probe_compare() -> int:
    """The round-2 no-flush probe of the half-split ring, rebuilt (knn.hip
    with -DGRID_ISA_PROBE: k_gram8<9, true, 1, 3>, results dropped so every
    MFMA is dead), against production k_gram8<0, true, 1, 3> from the same
    object: frontier errors, and the steady K loop's barriers and vmcnt waits
    per 6-step trip (compile only; nothing runs on a GPU)."""
    src = Path(__file__).resolve().parent.parent / "grid_amd" / "csrc"
    with tempfile.TemporaryDirectory() as td:
        obj = Path(td) / "knn_probe.o"
        subprocess.run(["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "--offload-arch=gfx950", "-fPIC",
                        "-ffp-contract=off", "-I" + str(src.parent.parent / "include"), "-DGRID_ISA_PROBE", "-c",
                        str(src / "knn.hip"), "-o", str(obj)], check=True, capture_output=True)
        funcs = {}
        for co in code_objects(str(obj)):
            funcs.update(parse_functions(disassemble(co)))
    res = check(funcs, "k_gram8<")
    rows = {}
    for name in ("k_gram8<0, true, 1, 3>", "k_gram8<9, true, 1, 3>"):
        v = res[name]
        ring = [l for l in v["loops"] if l["lds_dma"] == 36 and l["innermost"]]
        steady = min(ring, key=lambda l: l["vmcnt"])
        rows[name] = (v["errors"], steady["barriers_per_iter"], steady["vmcnt"], steady["mfma"], steady["scratch"])
        print(f"{name}: frontier errors {len(v['errors'])}; steady trip: barriers {steady['barriers_per_iter']}, "
              f"vmcnt {steady['vmcnt']}, lgkmcnt {steady['lgkmcnt']}, dma {steady['lds_dma']}, "
              f"mfma {steady['mfma']}, scratch {steady['scratch']}")
    (e0, b0, v0, _, _), (e9, b9, v9, _, _) = rows.values()
    same = not e0 and not e9 and b0 == b9 and v0 == v9
    print("same barrier / vmcnt skeleton" if same else "SKELETONS DIFFER")
    return 0 if same else 1


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("lib", nargs="?", default="grid_amd/_lib/libgridhip.so")
    ap.add_argument("--kernels", default="", help="comma-separated name substrings (default: every kernel "
                                                  "that has a barrier)")
    ap.add_argument("--json", action="store_true")
    ap.add_argument("--probe", action="store_true", help="rebuild the round-2 no-flush Gram probe and compare "
                                                         "its ISA skeleton with production")
    a = ap.parse_args()
    if a.probe:
        sys.exit(probe_compare())
    funcs = {}
    for co in code_objects(a.lib):
        funcs.update(parse_functions(disassemble(co)))
    res = check(funcs, a.kernels)
    bad = {k: v["errors"] for k, v in res.items() if v["errors"]}
    if a.json:
        print(json.dumps(res, indent=1))
    else:
        for k, v in sorted(res.items()):
            loops = "; ".join(f"loop@{l['head']}: {l['barriers_per_iter']} bar/iter, {l['vmcnt']} vmcnt, "
                              f"{l['lgkmcnt']} lgkm, {l['lds_dma']} dma, {l['mfma']} mfma" for l in v["loops"]
                              if l["s_barrier"])
            print(f"{'BAD ' if v['errors'] else 'ok  '}{k[:90]}: {v['barriers']} s_barrier"
                  + (f"; {loops}" if loops else ""))
            for e in v["errors"]:
                print(f"      {e}")
    print(f"{len(res)} kernels with barriers checked, {len(bad)} with errors", file=sys.stderr)
    sys.exit(1 if bad else 0)


if __name__ == "__main__":
    main()
