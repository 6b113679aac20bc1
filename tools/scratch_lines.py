"""Histogram of scratch (spill / private array) instructions of one kernel by source line.
usage: python tools/scratch_lines.py <kernel-symbol-substring>   (builds planner.hip device asm with line tables)"""
import collections, re, subprocess, sys
k = sys.argv[1] if len(sys.argv) > 1 else 'lane_reach_kernel'
src = 'armour-dev_amd/csrc/planner.hip'
subprocess.run(['/opt/rocm/bin/hipcc', '--offload-arch=gfx950', '-O3', '-std=c++17', '-ffp-contract=off', '--cuda-device-only',
                '-gline-tables-only', '-S', src, '-o', '/tmp/scratch_lines.s'], check=True, stderr=subprocess.DEVNULL)
files, cur, on = {}, None, False
cnt = collections.Counter()
for l in open('/tmp/scratch_lines.s'):
    m = re.match(r'\s*\.file\s+(\d+)\s+"([^"]*)"\s*(?:"([^"]*)")?', l)
    if m:
        files[m.group(1)] = (m.group(3) or m.group(2)).split('/')[-1]
        continue
    if l.startswith('_Z') and ':' in l:
        on = k in l
    if not on:
        continue
    m = re.match(r'\s*\.loc\s+(\d+)\s+(\d+)', l)
    if m:
        cur = (files.get(m.group(1), m.group(1)), int(m.group(2)))
    elif 'scratch_' in l:
        cnt[(cur, 'st' if 'store' in l else 'ld')] += 1
lines = {}
for (f, ln), kind in cnt:
    if f and f.endswith(('.h', '.hip')) and ln:
        try:
            lines[(f, ln)] = open(f'armour-dev_amd/csrc/{f}').read().split('\n')[ln - 1].strip()[:90]
        except OSError:
            pass
for key, v in sorted(cnt.items(), key=lambda z: -z[1])[:int(sys.argv[2]) if len(sys.argv) > 2 else 25]:
    (f, ln), kind = key
    print(f'{v:4d} {kind} {f}:{ln}  {lines.get((f, ln), "")}')
