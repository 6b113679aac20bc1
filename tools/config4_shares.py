"""Config 4 (BASELINE configs[3]: one fixed job of 256 worlds sharded over 8 GPUs) measured on one
MI355X: the step time of each rank's share (256 / N worlds for N = 1, 2, 4, 8), at 1-3 concurrent
planners, through bench.py's strong-scaling mode. The predicted 1 -> N speedup is t(256) / t(256/N)
(each rank plans its share with no data-path collective; the one all-gather of 80-byte records is
not included).

usage: python tools/config4_shares.py <out.txt> [steps]"""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
out = sys.argv[1]
steps = sys.argv[2] if len(sys.argv) > 2 else "10"
lines = ["# worlds-per-rank, planners, plans/s, ms/step: bench.py --total-worlds N --planners P (one MI355X)"]
best = {}
for share in (256, 128, 64, 32):
    for planners in (1, 2, 3):
        cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--total-worlds", str(share), "--planners", str(planners),
               "--steps", steps, "--warmup", "2", "--cpu-seconds", "0", "--no-extras"]
        r = subprocess.run(cmd, capture_output=True, text=True, timeout=600)
        if r.returncode != 0:
            raise SystemExit(r.stderr[-2000:])
        rec = json.loads(r.stdout.strip().splitlines()[-1])
        lines.append(f"{share} {planners} {rec['value']:.1f} {rec['ms_per_step']:.2f}")
        best[share] = min(best.get(share, 1e30), rec["ms_per_step"])
        print(lines[-1], flush=True)
for n, share in ((2, 128), (4, 64), (8, 32)):
    lines.append(f"# predicted 1 -> {n} GPUs: {best[256] / best[share]:.2f}x (best planner count per share: "
                 f"{best[256]:.2f} / {best[share]:.2f} ms)")
    print(lines[-1])
open(out, "w").write("\n".join(lines) + "\n")
