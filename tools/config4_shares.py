"""Config 4 (BASELINE configs[3]: one fixed job of 256 worlds sharded over 8 GPUs) measured on one
MI355X: the step time of each rank's share (256 / N worlds for N = 1, 2, 4, 8) through bench.py's
strong-scaling mode, as bench.py runs it by default (--planners 0: each rank times 1, 2 and 3
concurrent planners on its share during warmup and keeps the fastest) and, for reference, at each
fixed planner count. The predicted 1 -> N speedup is t(256) / t(256/N) with the default flags (each
rank plans its share with no data-path collective; the one all-gather of 80-byte records is not
included).

usage: python tools/config4_shares.py <out.txt> [steps]"""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
out = sys.argv[1]
steps = sys.argv[2] if len(sys.argv) > 2 else "10"
lines = ["# worlds-per-rank, planners, plans/s, ms/step: bench.py --total-worlds N [--planners P] (one MI355X);",
         "# 'default' = no --planners flag (the per-share calibration, chosen count and calibration times shown)"]
dflt = {}


def run(share, planners):
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--total-worlds", str(share),
           "--steps", steps, "--warmup", "2", "--cpu-seconds", "0", "--no-extras"]
    if planners:
        cmd += ["--planners", str(planners)]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=600)
    if r.returncode != 0:
        raise SystemExit(r.stderr[-2000:])
    return json.loads(r.stdout.strip().splitlines()[-1])


for share in (256, 128, 64, 32):
    rec = run(share, 0)
    cfg = rec["config"]
    dflt[share] = rec["ms_per_step"]
    lines.append(f"{share} default({cfg['planners_per_gpu']}) {rec['value']:.1f} {rec['ms_per_step']:.2f} "
                 f"calibration {cfg.get('planner_calibration_ms')}")
    print(lines[-1], flush=True)
    for planners in (1, 2, 3):
        rec = run(share, planners)
        lines.append(f"{share} {planners} {rec['value']:.1f} {rec['ms_per_step']:.2f}")
        print(lines[-1], flush=True)
for n, share in ((2, 128), (4, 64), (8, 32)):
    lines.append(f"# predicted 1 -> {n} GPUs with the default flags: {dflt[256] / dflt[share]:.2f}x "
                 f"({dflt[256]:.2f} / {dflt[share]:.2f} ms)")
    print(lines[-1])
open(out, "w").write("\n".join(lines) + "\n")
