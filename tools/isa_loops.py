"""Scratch (spill) traffic of a kernel's loops, from its assembly (development tool, build container).

Compile one kernel to assembly with line tables, e.g. the dense bundle reach kernel:
    printf '#include "reach_kernel.hip"\\n#include "lane_kernel.hip"\\nnamespace armour { namespace lane {\\n'\\
'template __global__ void lane_reach_kernel<LaneDense>(const RobotParams*, LaneArgs, ReachOut);\\n}}\\n' > /tmp/lane_only.hip
    hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -gline-tables-only --cuda-device-only -S \\
        -I armour-dev_amd/csrc -o /tmp/lane.s /tmp/lane_only.hip
then
    python tools/isa_loops.py /tmp/lane.s [SOURCE_FILE LAST_LINE]
lists the loops (back edges) with the most scratch_load / scratch_store instructions, and with
SOURCE_FILE and LAST_LINE (e.g. lane_engine.h and the line of `base += __popcll(km);`) the loops whose
last source line of that file is LAST_LINE: the simplify round loops, with their spill sites."""
import collections
import re
import sys

lines = open(sys.argv[1]).read().split("\n")
files, loc, cur, labels = {}, [None] * len(lines), None, {}
for i, l in enumerate(lines):
    m = re.match(r'\s*\.file\s+(\d+)\s+"([^"]*)"\s*"([^"]*)"', l)
    if m:
        files[m.group(1)] = m.group(3).split("/")[-1]
    m = re.match(r"\s*\.loc\s+(\d+)\s+(\d+)", l)
    if m:
        cur = (files.get(m.group(1), m.group(1)), int(m.group(2)))
    loc[i] = cur
    m = re.match(r"^(\.LBB\d+_\d+):", l)
    if m:
        labels[m.group(1)] = i
loops = []
for i, l in enumerate(lines):
    m = re.match(r"\s*s_(cbranch_\w+|branch)\s+(\.LBB\d+_\d+)", l)
    if m and m.group(2) in labels and labels[m.group(2)] < i:
        loops.append((labels[m.group(2)], i))


def count(a, b, what):
    return sum(what in x for x in lines[a:b + 1])


if len(sys.argv) > 3:
    src, last = sys.argv[2], int(sys.argv[3])
    for a, b in sorted(set(loops)):
        own = [loc[j][1] for j in range(a, b + 1) if loc[j] and loc[j][0] == src]
        if not own or max(own) != last:
            continue
        sites = collections.Counter(loc[a + k] for k, x in enumerate(lines[a:b + 1]) if "scratch_" in x)
        print(f"loop at asm line {a}: {b - a} lines, scratch loads {count(a, b, 'scratch_load')}, "
              f"stores {count(a, b, 'scratch_store')}, global loads {count(a, b, 'global_load')}, "
              f"flat {count(a, b, 'flat_')}; spill sites {dict(sites.most_common(5))}")
else:
    for a, b in sorted(loops, key=lambda ab: -count(ab[0], ab[1], "scratch_"))[:30]:
        print(f"loop at asm line {a}: {b - a} lines, scratch loads {count(a, b, 'scratch_load')}, "
              f"stores {count(a, b, 'scratch_store')}, flat {count(a, b, 'flat_')}")
