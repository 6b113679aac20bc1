"""fp64 VALU rate of eval_kernel from a rocprofv3 PMC pass (tools/gpu_prof_round.sh) and the kernel
trace of the same command: FLOPs = 64 x (ADD_F64 + MUL_F64 + TRANS_F64 + 2 FMA_F64) wave
instructions (every lane counted, an upper bound), against the MI355X fp64 vector peak.
usage: eval_valu.py <counter_collection.csv> <kernel_trace.csv> <out.json>"""
import csv
import json
import sys

PEAK_FP64_TFLOPS = 78.6  # MI355X fp64 vector peak, AMD spec sheet (not in MI355X_MICROARCH.md)
SIMDS = 256 * 4
XCDS = 8  # GRBM_GUI_ACTIVE comes summed over the 8 XCDs (per dispatch ~8 x the kernel's cycles)


def main():
    pmc, trace, out = sys.argv[1:4]
    per = {}
    for r in csv.DictReader(open(pmc)):
        if "eval_kernel" not in r.get("Kernel_Name", ""):
            continue
        d = per.setdefault(r["Dispatch_Id"], {})
        d[r["Counter_Name"]] = d.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    durs = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9 for r in csv.DictReader(open(trace))
            if "eval_kernel" in r["Kernel_Name"]]
    if not per or not durs:
        raise SystemExit("no eval_kernel rows")
    keys = sorted(next(iter(per.values())))
    avg = {k: sum(d.get(k, 0.0) for d in per.values()) / len(per) for k in keys}
    t = sorted(durs)[len(durs) // 2]
    flops = 64 * (avg.get("SQ_INSTS_VALU_ADD_F64", 0) + avg.get("SQ_INSTS_VALU_MUL_F64", 0)
                  + avg.get("SQ_INSTS_VALU_TRANS_F64", 0) + 2 * avg.get("SQ_INSTS_VALU_FMA_F64", 0))
    res = dict(kernel="eval_kernel_t<double>", dispatches=len(per), counters_per_dispatch=avg, median_duration_s=t,
               fp64_flops_per_dispatch=flops, fp64_tflops=flops / t / 1e12, peak_fp64_tflops=PEAK_FP64_TFLOPS,
               frac_of_fp64_peak=flops / t / 1e12 / PEAK_FP64_TFLOPS,
               valu_busy=(4 * avg["SQ_ACTIVE_INST_VALU"] / (SIMDS * avg["GRBM_GUI_ACTIVE"] / XCDS)
                          if avg.get("GRBM_GUI_ACTIVE") and avg.get("SQ_ACTIVE_INST_VALU") else None),
               mean_resident_waves=(4 * avg["SQ_WAVE_CYCLES"] / (avg["GRBM_GUI_ACTIVE"] / XCDS)
                                    if avg.get("GRBM_GUI_ACTIVE") else None),
               fp64_share_of_valu=(avg.get("SQ_INSTS_VALU_ADD_F64", 0) + avg.get("SQ_INSTS_VALU_MUL_F64", 0)
                                   + avg.get("SQ_INSTS_VALU_FMA_F64", 0) + avg.get("SQ_INSTS_VALU_TRANS_F64", 0))
                                  / avg["SQ_INSTS_VALU"],
               note="valu_busy = 4 x SQ_ACTIVE_INST_VALU (quad-cycles, summed over waves) / (1024 SIMDs x "
                    "GRBM_GUI_ACTIVE / 8 XCDs): the share of SIMD cycles with a VALU instruction in issue; "
                    "mean_resident_waves = 4 x SQ_WAVE_CYCLES / kernel cycles (4096 = 4 waves on every SIMD)")
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
