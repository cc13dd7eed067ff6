"""Static instruction profile of one k_paths instantiation between the SPT_MARK comments of a
-DSPT_STATIC_PROFILE build (analysis only: the markers constrain scheduling a little).

    python scripts/static_profile.py [extra hipcc -D flags ...]

Compiles the C2 shape-specialized flat kernel and the two BVH k_paths instantiations to assembly and
prints, per section of the step loop, the VALU / SALU / LDS / scalar-memory / vector-memory
instruction counts (the code the compiler placed after a marker, up to the next one in program
order; the sections of divergent branches interleave, so read the counts as the code size of each
part, not as executed instructions)."""
import collections
import os
import re
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
C2_SHAPE = 77445755138  # flat_shape_key of the Cornell box (spt_kernels.h)
# ... with C2's launch configuration baked in (jit_config_key: 8 bounces, RR depth 2, sky, fast division)
C2_SHAPE |= (1 << 37) | (8 << 38) | (2 << 44) | (1 << 50) | (1 << 52)
C2_SHAPE |= 7 << 53  # every axis group of the box is walls (flat_rect_bits)
INST = r"""#include "spt_kernels.hip"
namespace spt {
#define I(S, B, SH, W) template __global__ void k_paths<S, B, 0, SH, W>(const float4* __restrict__, const float4* __restrict__, \
    const float4* __restrict__, uint32_t, float4* __restrict__, unsigned long long* __restrict__, uint32_t* __restrict__, \
    uint32_t* __restrict__, ShadeParams, CameraParams, uint32_t, ChunkPlan, NeeParams);
I(false, false, %dull, 0)
}
""" % C2_SHAPE


def classify(op):
    if op.startswith("v_"):
        return "valu"
    if op.startswith(("s_load", "s_buffer_load")):
        return "smem"
    if op.startswith("s_waitcnt") or op.startswith("s_nop"):
        return "wait"
    if op.startswith("s_"):
        return "salu"
    if op.startswith("ds_"):
        return "lds"
    if op.startswith(("global_", "buffer_", "flat_", "scratch_")):
        return "vmem"
    return "other"


def main():
    flags = sys.argv[1:]
    with tempfile.TemporaryDirectory() as td:
        src = os.path.join(td, "inst.hip")
        open(src, "w").write(INST)
        asm = os.path.join(td, "inst.s")
        cmd = ["/opt/rocm/bin/hipcc", "-O3", "-fno-slp-vectorize", "-ffp-contract=off", "-fno-fast-math",
               "-std=c++17", "--offload-arch=gfx950", "-fno-gpu-rdc", "-I" + os.path.join(ROOT, "include"),
               "-I" + os.path.join(ROOT, "software-path-tracer_amd", "csrc"), "--cuda-device-only", "-S",
               "-DSPT_STATIC_PROFILE", *flags, "-o", asm, src]
        subprocess.run(cmd, check=True, stderr=subprocess.DEVNULL)
        lines = open(asm).read().split("\n")
    for kname in ("_ZN3spt7k_pathsILb0ELb0ELi0ELm%dELi0E" % C2_SHAPE, "_ZN3spt7k_pathsILb0ELb1ELi0ELm0ELi8E",
                  "_ZN3spt7k_pathsILb0ELb1ELi0ELm0ELi0E"):
        on, sec = False, "prologue"
        cnt = collections.defaultdict(collections.Counter)
        for ln in lines:
            if re.match(r"^" + kname + r".*:", ln):
                on = True
                continue
            if not on:
                continue
            if ln.startswith(".Lfunc_end"):
                break
            m = re.search(r"SPT_MARK (\w+)", ln)
            if m:
                sec = m.group(1)
                continue
            s = ln.strip()
            if not s or s.startswith((";", ".")) or s.endswith(":"):
                continue
            cnt[sec][classify(s.split()[0])] += 1
        if not cnt:
            continue
        print(kname)
        tot = sum(c["valu"] for c in cnt.values())
        for sec, c in cnt.items():
            print(f"  {sec:26s} valu {c['valu']:5d} ({100.0 * c['valu'] / max(tot, 1):4.1f} %)  salu {c['salu']:4d}  "
                  f"lds {c['lds']:3d}  smem {c['smem']:3d}  vmem {c['vmem']:3d}  wait {c['wait']:3d}")


if __name__ == "__main__":
    main()
