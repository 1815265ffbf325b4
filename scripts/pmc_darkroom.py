"""Summarise the DarkRoom kernel's PMC passes (scripts/profile_darkroom.sh) into
profiles/pmc_rollout_darkroom.json: MFMA pipe busy fraction, executed MFMAs,
effective clock, HBM fetch (FETCH_SIZE x2, gfx950 calibration)."""
import csv
import json
import sys


def counters(path, kernel="rollout_darkroom_kernel"):
    out = {}
    for r in csv.DictReader(open(path)):
        if kernel in r["Kernel_Name"]:
            out.setdefault(r["Counter_Name"], []).append(float(r["Counter_Value"]))
    return {k: sum(v) / len(v) for k, v in out.items()}


def main(stats, mfma, fetch, out):
    st = [r for r in csv.DictReader(open(stats)) if "rollout_darkroom" in r["Name"]][0]
    ns = float(st["AverageNs"])
    v = counters(mfma)
    res = {"kernel": "rollout_darkroom_kernel",
           "workload": "config 3: 4096 tasks, Heps=40, horizon=H=100 (one launch = one online eval)",
           "kernel_ms_avg_trace": ns / 1e6, "GRBM_GUI_ACTIVE": v["GRBM_GUI_ACTIVE"],
           "SQ_VALU_MFMA_BUSY_CYCLES": v["SQ_VALU_MFMA_BUSY_CYCLES"],
           "effective_clock_GHz": v["GRBM_GUI_ACTIVE"] / 8 / (ns * 1e-9) / 1e9,
           "mfma_pipe_busy_frac": v["SQ_VALU_MFMA_BUSY_CYCLES"] / (1024 * v["GRBM_GUI_ACTIVE"] / 8),
           "note": "busy cycles summed over the 1024 SIMDs: 16 per v_mfma_f32_16x16x32_f16 (every product of the "
                   "blocks as fp16 two-part split products, three per K=32 tile, end of round 2); "
                   "GRBM_GUI_ACTIVE is summed over 8 XCDs"}
    if fetch:
        res["hbm_fetch_bytes_corrected"] = 2 * counters(fetch)["FETCH_SIZE"] * 1024
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main(*sys.argv[1:4], sys.argv[4])
