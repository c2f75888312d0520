"""Static instruction counts of a kernel in a csrc source (device-only ISA, shipped flags), for
quick before/after checks of VALU-trimming edits on the CPU box.

    python tools/isa_count.py [swarm.hip] [k_lattice_filterILb1] [-DFOO=1 ...]
"""
import os
import re
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "cbf_amd", "csrc")


def counts(src="swarm.hip", kernel="k_lattice_filterILb1", defines=()):
    with tempfile.TemporaryDirectory() as td:
        out = os.path.join(td, "k.s")
        cmd = ["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-ffp-contract=off",
               "-I", os.path.join(ROOT, "include"), "-I", CSRC, "--cuda-device-only", "-S", "-x", "hip",
               os.path.join(CSRC, src), "-o", out] + list(defines)
        subprocess.run(cmd, check=True, stderr=subprocess.DEVNULL)
        lines = open(out).read().split("\n")
    start = next(i for i, l in enumerate(lines) if re.match(r"^_Z\S*" + kernel + r"\S*:", l))
    end = next(i for i in range(start, len(lines)) if lines[i].startswith(".Lfunc_end"))  # (several s_endpgm)
    body = lines[start:end]
    res = {"valu": sum(1 for l in body if re.match(r"\s+v_", l)),
           "salu": sum(1 for l in body if re.match(r"\s+s_", l)),
           "vmem": sum(1 for l in body if re.match(r"\s+(global|buffer)_", l)),
           "lds": sum(1 for l in body if re.match(r"\s+ds_", l))}
    sym = re.match(r"^(\S+):", lines[start]).group(1)
    for l in lines:
        m = re.match(r"\s*\.set " + re.escape(sym) + r"\.(num_vgpr|private_seg_size), (\d+)", l)
        if m:
            res[m.group(1)] = int(m.group(2))
    return res


if __name__ == "__main__":
    a = sys.argv[1:]
    src = a[0] if a and not a[0].startswith("-") else "swarm.hip"
    kern = a[1] if len(a) > 1 and not a[1].startswith("-") else "k_lattice_filterILb1"
    print(counts(src, kern, [x for x in a if x.startswith("-D")]))
