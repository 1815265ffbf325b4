"""Summarise the DarkRoom kernel's PMC passes (scripts/profile_darkroom.sh) into
profiles/pmc_rollout_darkroom.json: MFMA pipe busy fraction, effective clock, HBM fetch
(FETCH_SIZE x2, gfx950 calibration), and where the wave cycles go (SQ_WAIT_ANY = parked at
s_waitcnt / barriers, SQ_WAIT_INST_ANY = issue stalls on dependencies / pipes, SQ_ACTIVE_INST_*
= issuing; the three are disjoint and sum to SQ_WAVE_CYCLES), with the instruction mix.
Usage: python scripts/pmc_darkroom.py <prof_dir> <out.json>"""
import csv
import glob
import json
import os
import sys


def counters(d, kernel="rollout_darkroom_kernel"):
    out = {}
    for path in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(path)):
            if kernel in r["Kernel_Name"]:
                out.setdefault(r["Counter_Name"], []).append(float(r["Counter_Value"]))
    return {k: sum(v) / len(v) for k, v in out.items()}  # per dispatch


def main(prof, out):
    stats = glob.glob(os.path.join(prof, "trace", "**", "*kernel_stats.csv"), recursive=True)[0]
    st = [r for r in csv.DictReader(open(stats)) if "rollout_darkroom" in r["Name"]][0]
    ns = float(st["AverageNs"])
    c = {}
    for name in ("mfma", "mem", "stall", "insts", "lds"):
        c.update(counters(os.path.join(prof, f"pmc_{name}")))
    simd_cycles = 1024 * c["GRBM_GUI_ACTIVE"] / 8
    res = {"kernel": "rollout_darkroom_kernel",
           "workload": "config 3: 4096 tasks, Heps=40, horizon=H=100 (one launch = one online eval)",
           "kernel_ms_avg_trace": ns / 1e6, "counters_per_dispatch": c,
           "effective_clock_GHz": c["GRBM_GUI_ACTIVE"] / 8 / (ns * 1e-9) / 1e9,
           "mfma_pipe_busy_frac": c["SQ_VALU_MFMA_BUSY_CYCLES"] / simd_cycles,
           "hbm_fetch_bytes_corrected": 2 * c["FETCH_SIZE"] * 1024}
    wc = c.get("SQ_WAVE_CYCLES")
    if wc:
        res["wave_cycle_fractions"] = {k: c[k] / wc for k in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY",
                                                            "SQ_ACTIVE_INST_VALU", "SQ_ACTIVE_INST_LDS",
                                                            "SQ_ACTIVE_INST_SCA", "SQ_ACTIVE_INST_MISC") if k in c}
        res["wave_cycle_fractions"]["SQ_WAIT_INST_LDS"] = c.get("SQ_WAIT_INST_LDS", 0) / wc
    if "SQ_INSTS_VALU" in c:
        res["instruction_mix_per_dispatch"] = {k: c[k] for k in c if k.startswith("SQ_INSTS")}
    if "SQ_LDS_IDX_ACTIVE" in c and c["SQ_LDS_IDX_ACTIVE"]:
        res["lds_bank_conflict_frac_of_lds_cycles"] = c["SQ_LDS_BANK_CONFLICT"] / c["SQ_LDS_IDX_ACTIVE"]
    if "SQ_VALU_MFMA_COEXEC_CYCLES" in c:
        res["valu_mfma_coexec_frac"] = c["SQ_VALU_MFMA_COEXEC_CYCLES"] / simd_cycles
    if "SQ_ACTIVE_INST_VALU" in c:
        # the issue roofline: SIMD cycles with VALU issue (quad-cycles x 4, summed over the waves of
        # a SIMD, which issue one VALU instruction at a time), with the MFMA pipe busy, and with
        # either (the co-executed cycles counted once)
        valu = 4 * c["SQ_ACTIVE_INST_VALU"] / simd_cycles
        res["simd_valu_issue_frac"] = valu
        res["simd_valu_or_mfma_busy_frac"] = valu + res["mfma_pipe_busy_frac"] - res.get("valu_mfma_coexec_frac", 0)
    if wc:
        res["avg_waves_per_simd"] = 4 * wc / simd_cycles
    res["note"] = ("SQ_WAVE_CYCLES / SQ_WAIT_* / SQ_ACTIVE_INST_* count quad-cycles (guide, cycle constants); "
                   "SQ_VALU_MFMA_BUSY_CYCLES counts cycles, summed over the 1024 SIMDs (16 per "
                   "v_mfma_f32_16x16x32_f16); GRBM_GUI_ACTIVE is summed over the 8 XCDs")
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
