"""Static instruction budget of one render kernel, by source region.

    python tools/valu_budget.py [asm.s] [kernel-symbol-substring]

The assembly comes from the package's device flags plus -g (line tables only; the instruction
stream is the same schedule the library runs, up to debug-induced noise):

    hipcc <Makefile HIPFLAGS> -g --cuda-device-only -S csrc/pt_device.hip -o pt_device_g.s

Every instruction of the kernel is attributed to the source line of its last `.loc`: inlined
helpers keep their own lines (wideHits, primHitAny, onUnitSphere, sampleStream, ...), macro
expansions (PT_TAKE_TASKS, PT_NEW_PATH, PT_BEGIN_RAY) the line that invokes them.  Lines are
grouped into regions: the helper function that contains them, or -- inside renderKernelWF itself
-- the step the line belongs to (the `// ---- NODE / LEAF / SHADE` markers).  Counts are STATIC
(instructions in the code, once each); the dynamic share of a region is its count times how often
its code runs (iterations per step kind from a PT_ITER_STATS run, loop trips), which
DESIGN.md section 11 works out next to this table.
"""
import collections
import os
import re
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(REPO, "path-tracer-cuda-opengl_amd", "csrc", "pt_device.hip")


GENERIC = {"add", "sub", "mul", "scale", "neg", "dot3", "cross3", "len2", "divs", "normalize3", "xyz", "f3",
           "ld3", "shlOpaque", "mul80", "mul48", "pt_math.hpp", "__clang_hip_math.h", "amd_warp_functions.h",
           "amd_device_functions.h", "amd_hip_atomic.h", "amd_hip_vector_types.h", "?", "__launch_bounds__",
           "kargs", "ldScene", "rawRsrc", "bload4", "file scope"}


NOT_NAMES = {"__launch_bounds__", "__attribute__", "amdgpu_waves_per_eu", "kWavesPerEU", "if", "for", "while",
             "return", "sizeof", "decltype", "static_assert"}


def classify(op: str) -> str:
    if op.startswith(("buffer_", "global_", "flat_", "scratch_")):
        return "vmem"
    if op.startswith("ds_"):
        return "lds"
    if op.startswith("s_load") or op.startswith("s_buffer_load"):
        return "smem"
    if op.startswith(("s_cbranch", "s_branch")):
        return "branch"
    if op.startswith("s_waitcnt") or op in ("s_nop", "s_setprio", "s_sleep"):
        return "wait"
    if op.startswith("s_"):
        return "salu"
    if op.startswith("v_"):
        return "valu"
    return "other"


def source_regions():
    """line -> region: the innermost enclosing device function (by definition line), and inside the
    render kernel its NODE / LEAF / SHADE steps and macro definitions."""
    lines = open(SRC).read().split("\n")
    fdef = re.compile(r"^(?:template <[^>]*>\s*)?(?:__global__|__device__|static|inline|constexpr).*?\b(\w+)\s*\(")
    region = {}
    cur = saved = "file scope"
    for i, ln in enumerate(lines, start=1):
        m = fdef.match(ln)
        if m and not ln.rstrip().endswith(";"):
            names = [n for n in re.findall(r"\b(\w+)\s*\(", ln) if n not in NOT_NAMES]
            if names:
                cur = names[0]
        mm = re.match(r"^#define (PT_\w+)\(", ln)
        if mm:
            saved, cur = cur, mm.group(1)
        if cur.startswith("PT_") and not ln.rstrip().endswith("\\"):
            region[i] = cur   # the macro's last line; the enclosing region resumes after it
            cur = saved
            continue
        if cur == "renderKernelWF" or cur.startswith("renderKernelWF:"):
            s = ln.strip()
            if "// ---" in s and any(k in s for k in ("NODE", "LEAF", "SHADE")):
                cur = "renderKernelWF:" + next(k for k in ("NODE", "LEAF", "SHADE") if k in s)
            elif s.startswith("for (;;) {") and cur == "renderKernelWF":
                cur = "renderKernelWF:loop head"
        if ln.startswith("#define PT_") and not ln.startswith("#define PT_DIAG_ADD") and "(" in ln.split()[1]:
            pass
        region[i] = cur
    return region


def main() -> None:
    asm = sys.argv[1] if len(sys.argv) > 1 else "/tmp/isa/pt_device_g.s"
    want = sys.argv[2] if len(sys.argv) > 2 else "renderKernelWFILi8ELb1ELb1ELb0E"
    text = open(asm).read().split("\n")
    files = {}
    start = None
    for i, ln in enumerate(text):
        m = re.match(r'\s*\.file\s+(\d+)\s+"([^"]*)"\s+"([^"]*)"', ln)
        if m:
            files[int(m.group(1))] = os.path.join(m.group(2), m.group(3))
        if start is None and ln.startswith("_Z") and want in ln and ln.rstrip().endswith(want + "EEEvNS_12RenderParamsE:") or \
                (start is None and ln.startswith("_Z") and want in ln and ln.split(":")[0].endswith("E") and ln.endswith(":")):
            start = i
    if start is None:
        for i, ln in enumerate(text):
            if re.match(r"^_Z\S*" + re.escape(want) + r"\S*:", ln):
                start = i
                break
    assert start is not None, want
    region = source_regions()
    per_line = collections.defaultdict(collections.Counter)
    per_region = collections.defaultdict(collections.Counter)
    total = collections.Counter()
    cur = ("?", 0)
    # (instructions of generic helpers -- vector arithmetic, reciprocals, warp intrinsics, code
    # without a line -- take the region of the nearest distinctive instruction of their basic block:
    # the .loc lines name only the innermost inlined function, not its caller)
    blocks, blk = [], []
    for ln in text[start + 1:]:
        if ln.startswith(".Lfunc_end"):
            break
        s = ln.strip()
        m = re.match(r"\.loc\s+(\d+)\s+(\d+)", s)
        if m:
            cur = (files.get(int(m.group(1)), "?"), int(m.group(2)))
            continue
        if s.endswith(":") and not s.startswith(";"):
            if blk:
                blocks.append(blk)
            blk = []
            continue
        if not s or s.startswith((".", ";")):
            continue
        op = s.split()[0]
        c = classify(op)
        total[c] += 1
        f, line = cur
        reg = region.get(line, "?") if f.endswith("pt_device.hip") else os.path.basename(f)
        if reg in GENERIC or line == 0:
            reg = None
        blk.append((c, reg, (os.path.basename(f), line)))
        if c in ("branch",) and (op.startswith("s_branch") or op.startswith("s_cbranch")):
            blocks.append(blk)
            blk = []
    if blk:
        blocks.append(blk)
    prev = "(no source line)"
    for b in blocks:   # a block of generic code only: the region of the code laid out before it
        last = next((r for _, r, _ in b if r), prev)
        for c, r, key in b:
            if r:
                last = r
            per_region[r or last][c] += 1
            per_line[key][c] += 1
        prev = last
    print(f"kernel {want}: " + ", ".join(f"{k} {v}" for k, v in total.most_common()))
    print(f"{'region':40s} {'VALU':>6s} {'SALU':>6s} {'VMEM':>5s} {'LDS':>4s} {'br':>4s}")
    for reg, c in sorted(per_region.items(), key=lambda kv: -kv[1]["valu"]):
        print(f"{reg:40s} {c['valu']:6d} {c['salu']:6d} {c['vmem']:5d} {c['lds']:4d} {c['branch']:4d}")
    print("\ntop source lines by static VALU:")
    src = open(SRC).read().split("\n")
    for (f, line), c in sorted(per_line.items(), key=lambda kv: -kv[1]["valu"])[:45]:
        txt = src[line - 1].strip()[:70] if f == "pt_device.hip" and 0 < line <= len(src) else ""
        print(f"  {f}:{line:<5d} {c['valu']:4d}  {txt}")


if __name__ == "__main__":
    main()
