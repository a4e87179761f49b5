#!/usr/bin/env python3
"""Instruction counts of the packet walk's BLAS loops from the ISA ("count the VALU and SALU
instructions per BLAS node visit and per triangle test from the ISA").

Compiles csrc/rt_trace.hip to gfx950 assembly with the Makefile's flags (or reads --asm), cuts out one
k_trace_frame_packet instantiation (default: the C2 kernel <1,false,1,1,false,false>), finds its BLAS walk loops
(the loop headers are the blocks holding the six octant-row s_load_dwordx4 of packet_blas_walk) and tags every
basic block of each loop:
  node       the loop header: node record loads, the 4 x 4 slab tests, the four ballots, the entered mask
  choice     the nearest-first choice of a closest-hit node with >= 2 entered internal children (keys, readlane)
  push       the stack push of the remaining entered children (one v_writelane)
  pop        the pop of the top entry (v_readlane, slot bookkeeping, v_writelane)
  tri-load   a triangle slot's record load (s_mul ... 48, s_load_dwordx8 / x4) and the 1 / det range check
  tri-test   the rest of Moller-Trumbore and the (t, instance, primitive) acceptance
  tri-take   the hit record update of the lanes that accept (exec-masked v_movs)
  tri-div    the IEEE division's slow path (det outside the fast reciprocal's range: rare)
  glue       branches, slot checks and the structurizer's flag blocks between them
Per tag it prints VALU / SALU / SMEM / s_nop / s_waitcnt / branch counts (one instance of each block), and the
per-visit totals of the common paths.

  python3 tools/isa_count.py [--asm FILE.s] [--kernel MANGLED] [--blocks]
"""
import argparse
import collections
import os
import re
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(ROOT, "realtimeraytracing_gradproject_amd", "csrc", "rt_trace.hip")
FLAGS = ["--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-ffp-contract=off", "-munsafe-fp-atomics",
         "-fno-slp-vectorize", "-mllvm", "-structurizecfg-skip-uniform-regions=1"]  # Makefile HIPFLAGS + TRACEFLAGS
C2_KERNEL = ("_ZN2rt12_GLOBAL__N_121k_trace_frame_packet8ILi1ELb0ELi1ELi1ELb0ELb0EEEvNS_9SceneViewENS_11FrameParams"
             "EPKjPjP15HIP_vector_typeIfLj4EEPy")
ROW_LOAD = re.compile(r"^s_load_dwordx4 s\[\d+:\d+\], s\[\d+:\d+\], s\d+$")
KINDS = ["valu", "salu", "smem", "nop", "wait", "br", "vmem", "lds"]


def kind(op):
    if op == "s_nop":
        return "nop"
    if op.startswith("s_waitcnt"):
        return "wait"
    if op.startswith("s_cbranch") or op == "s_branch":
        return "br"
    if op.startswith(("s_load", "s_buffer_load")):
        return "smem"
    if op.startswith("s_"):
        return "salu"
    if op.startswith("v_"):
        return "valu"
    if op.startswith(("global_", "buffer_", "flat_")):
        return "vmem"
    if op.startswith("ds_"):
        return "lds"
    return "other"


def compile_asm(out):
    cmd = ["/opt/rocm/bin/hipcc"] + FLAGS + ["--cuda-device-only", "-S", "-o", out, SRC]
    subprocess.run(cmd, check=True, capture_output=True, text=True)


def kernel_lines(asm, name):
    lines = open(asm).read().split("\n")
    start = next(i for i, l in enumerate(lines) if l.startswith(name + ":"))
    end = start + 1
    while not lines[end].strip().startswith("s_endpgm"):
        end += 1
    return lines[start:end + 1]


def blocks_of(lines):
    """[(label, loop_header or None, [instruction lines])] in program order."""
    out, cur = [], None
    for l in lines:
        t = l.strip()
        m = re.match(r"(\.LBB\d+_\d+):|; (%bb\.\d+):", t)
        if m:
            hdr = re.search(r"Header=BB(\d+_\d+)", t)
            is_hdr = "Inner Loop Header" in l or "Loop Header" in l
            cur = {"label": m.group(1) or m.group(2), "loop": hdr.group(1) if hdr else None, "ins": [],
                   "header": is_hdr}
            out.append(cur)
            continue
        if cur is None or not t or t.startswith((";", ".")):
            continue
        cur["ins"].append(t)
    return out


def tag(b):
    ops = [i.split()[0] for i in b["ins"]]
    text = "\n".join(b["ins"])
    if sum(1 for i in b["ins"] if ROW_LOAD.match(i)) == 6:
        return "node"
    if "v_div_scale_f32" in ops:
        return "tri-div"
    if "v_readlane_b32" in ops and "s_ff1_i32_b32" in ops:
        return "pop"
    if ("v_bfe_i32" in ops or "v_min3_u32" in ops) and "v_readlane_b32" in ops:
        return "choice"
    if "v_writelane_b32" in ops:
        return "push"
    if re.search(r"s_mul_i32 s\d+, s\d+, 48", text):
        return "tri-load"
    if ops.count("v_mul_f32_e32") + ops.count("v_fmac_f32_e32") >= 10:
        return "tri-test"
    if ops and all(o == "v_mov_b32_e32" for o in ops) and len(ops) >= 4:
        return "tri-take"
    return "glue"


def count(ins):
    c = collections.Counter(kind(i.split()[0]) for i in ins)
    return {k: c.get(k, 0) for k in KINDS if c.get(k, 0)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--asm", help="gfx950 assembly of rt_trace.hip (default: compile it to /tmp)")
    ap.add_argument("--kernel", default=C2_KERNEL)
    ap.add_argument("--blocks", action="store_true", help="print every block of the loops")
    a = ap.parse_args()
    asm = a.asm
    if not asm:
        asm = "/tmp/rt_trace_isa_count.s"
        compile_asm(asm)
    blocks = blocks_of(kernel_lines(asm, a.kernel))
    headers = [b for b in blocks if tag(b) == "node"]
    for h in headers:
        hid = h["label"].replace(".LBB", "")
        loop = [b for b in blocks if b is h or b["loop"] == hid]
        walk = "closest-hit" if any(tag(b) == "choice" for b in loop) else "any-hit"
        print(f"== BLAS walk loop {h['label']} ({walk}): {len(loop)} blocks")
        per = collections.defaultdict(collections.Counter)
        for b in loop:
            t = tag(b)
            c = count(b["ins"])
            per[t].update(c)
            if a.blocks:
                print(f"   {b['label']:12s} {t:9s} {c}")
        for t in ["node", "choice", "push", "pop", "tri-load", "tri-test", "tri-take", "tri-div", "glue"]:
            if t in per:
                print(f"   {t:9s} " + " ".join(f"{k}={per[t][k]}" for k in KINDS if per[t][k]))
        # per-visit totals: a triangle test = its load + test blocks (x4 slots unrolled: one slot's worth)
        nt = max(1, sum(1 for b in loop if tag(b) == "tri-test"))
        tri = collections.Counter()
        for t in ("tri-load", "tri-test"):
            tri.update(per[t])
        print(f"   per triangle test (one of {nt} unrolled slots, no take): "
              + " ".join(f"{k}={tri[k] // nt}" for k in KINDS if tri[k]))
    if not headers:
        print("no BLAS walk loop found (the octant-row loads moved?)", file=sys.stderr)
        return 1
    return 0


if __name__ == "__main__":
    sys.exit(main())
