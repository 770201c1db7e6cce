"""Instruction counts of one kernel's hot loops from an object built by fet-ode_amd/csrc/Makefile.

usage: python tools/diag/isa_count.py <obj.o> <kernel-substring> [--loops]
       python tools/diag/isa_count.py --marks <src.hip> <kernel-substring> [-Dextra ...]

Extracts the gfx950 code object from the offload bundle (in /tmp), disassembles the kernel,
finds its backward branches (loops) and prints, per loop, the instruction count and a class
histogram: transcendental, packed fp32, other VALU, DPP, LDS, SALU/branch, s_nop, waitcnt.
A static count (no trip counts): for the rk4 fused kernels each loop body is one rk4 step
(four inlined evaluations)."""
import collections
import os
import re
import subprocess
import sys

LLVM = "/opt/rocm/lib/llvm/bin"


def extract(obj):
    import shutil
    out = f"/tmp/isa_{os.getpid()}"
    os.makedirs(out, exist_ok=True)
    src = os.path.join(out, "k.o")
    shutil.copy(obj, src)
    # llvm-objdump --offloading writes the bundle's entries next to its input
    subprocess.run([f"{LLVM}/llvm-objdump", "--offloading", src], check=True, capture_output=True)
    co = src + ".0.hipv4-amdgcn-amd-amdhsa--gfx950"
    text = subprocess.run([f"{LLVM}/llvm-objdump", "-d", co], check=True, capture_output=True, text=True).stdout
    shutil.rmtree(out, ignore_errors=True)
    return text


def classify(op):
    if re.match(r"v_(exp|rcp|log|rsq|sqrt|sin|cos)_f32", op):
        return "trans"
    if op.startswith("v_pk_"):
        return "packed"
    if "_dpp" in op or op.startswith("v_permlane"):
        return "dpp"
    if op.startswith("ds_"):
        return "lds"
    if op.startswith("s_nop"):
        return "nop"
    if op.startswith("s_waitcnt"):
        return "wait"
    if op.startswith("s_"):
        return "salu"
    if op.startswith("v_"):
        return "valu"
    if op.startswith(("global_", "buffer_", "flat_", "scratch_")):
        return "vmem"
    return "other"


def main():
    obj, name = sys.argv[1], sys.argv[2]
    text = extract(obj)
    lines = text.splitlines()
    start = None
    for i, l in enumerate(lines):
        if re.match(r"^[0-9a-f]+ <.*>:$", l):
            if start is not None:
                end = i
                break
            if name in l:
                start = i
    else:
        end = len(lines)
    body = lines[start:end]
    print(body[0])
    insts = []   # (addr, op, text)
    for l in body[1:]:
        m = re.match(r"\s+(\w+)(.*?)//\s*([0-9A-F]+):", l)
        if m:
            insts.append((int(m.group(3), 16), m.group(1), l))
    addr_idx = {a: i for i, (a, _, _) in enumerate(insts)}
    loops = []
    for i, (a, op, l) in enumerate(insts):
        if op.startswith("s_cbranch") or op == "s_branch":
            m = re.search(r"<[^>]*\+0x([0-9a-f]+)>", l)
            if m:
                tgt = int(m.group(1), 16) + insts[0][0] - 0  # offsets are from the symbol start
                # symbol start = address of the first instruction
                if tgt <= a and tgt in addr_idx and i - addr_idx[tgt] > 200:
                    loops.append((addr_idx[tgt], i))
    tot = collections.Counter(classify(op) for _, op, _ in insts)
    print("kernel:", len(insts), dict(tot))
    # innermost large loops: drop any range that contains another one
    loops = sorted(set(loops))
    loops = [(lo, hi) for lo, hi in loops
             if not any((lo2, hi2) != (lo, hi) and lo <= lo2 and hi2 <= hi for lo2, hi2 in loops)]
    for lo, hi in loops:
        c = collections.Counter(classify(op) for _, op, _ in insts[lo:hi + 1])
        print(f"loop [{lo}, {hi}] {hi - lo + 1} instructions:", dict(sorted(c.items())))
        if "--loops" in sys.argv:
            ops = collections.Counter(op for _, op, _ in insts[lo:hi + 1])
            print("   ", ", ".join(f"{k} {v}" for k, v in ops.most_common(40)))


if __name__ == "__main__" and "--marks" not in sys.argv:
    main()


def marks(src, name, extra=()):
    """Per-phase counts from a device-only -S build with FETODE_ISA_MARKERS: the instructions between
    consecutive '; MARK <phase>' comments of kernel `name`, averaged over the phase's occurrences
    (the phases of one fused evaluation: X_FEAT, EDGES0, H_FEAT, EDGES1, END)."""
    out = f"/tmp/isa_marks_{os.getpid()}.s"
    subprocess.run(["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "--offload-arch=gfx950", "-ffp-contract=off",
                    "--cuda-device-only", "-S", "-DFETODE_ISA_MARKERS", *extra, "-o", out, src], check=True)
    lines = open(out).read().splitlines()
    os.remove(out)
    inside, cur = False, None
    per = collections.defaultdict(collections.Counter)
    occ = collections.Counter()
    for l in lines:
        if re.match(r"^\S+:", l) and not l.startswith((".", "$")):
            inside = name in l
            cur = None
            continue
        if not inside:
            continue
        m = re.search(r"; MARK (\w+)", l)
        if m:
            cur = m.group(1)
            occ[cur] += 1
            continue
        m = re.match(r"\s+([a-z]\w+)", l)
        if m and cur and not l.strip().startswith((";", ".")):
            per[cur][classify(m.group(1))] += 1
    for k in per:
        n = occ[k]
        c = {a: round(b / n, 1) for a, b in sorted(per[k].items())}
        print(f"{k:8s} x{n:3d}  total {sum(per[k].values()) / n:6.1f}  {c}")


if __name__ == "__main__" and "--marks" in sys.argv:
    # python tools/diag/isa_count.py --marks <src.hip> <kernel-substring> [-Dextra ...]
    a = [x for x in sys.argv[1:] if x != "--marks"]
    marks(a[0], a[1], a[2:])
