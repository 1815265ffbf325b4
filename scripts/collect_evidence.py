"""Copy one evidence pass (scripts/gpu_evidence.sh TAG, merged into gpurun_out/) into profiles/TAG/
and regenerate the PMC summaries bench.py reads for the roofline `traffic`:
profiles/pmc_rollout_bandit.json (config 2), profiles/pmc_rollout_linear.json (config 4's shard) and
profiles/pmc_rollout_darkroom.json (config 3).

    python scripts/collect_evidence.py r6a
"""
import json
import os
import shutil
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "scripts"), ROOT]


def cp(src, dst):
    if os.path.exists(src):
        os.makedirs(os.path.dirname(dst), exist_ok=True)
        shutil.copy(src, dst)
        return True
    return False


def strip_drm(src, dst):
    """copy a JSON output without the libdrm warning line the box prints on stderr"""
    if os.path.exists(src):
        lines = [ln for ln in open(src) if "amdgpu.ids" not in ln]
        open(dst, "w").write("".join(lines))


def main(tag):
    g = os.path.join(ROOT, "gpurun_out")
    p = os.path.join(ROOT, "profiles", tag)
    os.makedirs(p, exist_ok=True)
    cp(f"{g}/provenance_{tag}.txt", f"{p}/provenance.txt")
    cp(f"{g}/gpu_tests.log", f"{p}/gpu_tests.log.txt")
    cp(f"{g}/smoke.log", f"{p}/smoke.log.txt")
    strip_drm(f"{g}/bench_{tag}.json", f"{p}/bench.json")
    strip_drm(f"{g}/logit_err_{tag}.json", f"{p}/dr_logit_error.json")
    # traces: per-kernel stats of the three workloads
    cp(f"{g}/prof_{tag}/trace/run_kernel_stats.csv", f"{p}/bandit_kernel_stats.csv")
    cp(f"{g}/prof_dr_{tag}/trace/run_kernel_stats.csv", f"{p}/darkroom_kernel_stats.csv")
    cp(f"{g}/prof45_{tag}/lin_trace/run_kernel_stats.csv", f"{p}/linear_c4_shard_kernel_stats.csv")
    cp(f"{g}/prof45_{tag}/c5_trace/run_kernel_stats.csv", f"{p}/darkroom_c5_shard_kernel_stats.csv")
    # PMC passes
    for name in ("mfma", "mem", "stall", "insts", "lds"):
        cp(f"{g}/prof_dr_{tag}/pmc_{name}/run_counter_collection.csv", f"{p}/darkroom_pmc_{name}.csv")
    for src, dst in (("pmc_fetch", "pmc_fetch_size.csv"), ("pmc_write", "pmc_write_size.csv"),
                     ("pmc_l2", "pmc_tcc_hit_miss.csv")):
        cp(f"{g}/prof_{tag}/{src}/run_counter_collection.csv", f"{p}/{dst}")
        cp(f"{g}/prof45_{tag}/lin_{src}/run_counter_collection.csv", f"{p}/linear_{dst}")
    import bench
    import pmc_darkroom
    import pmc_summary
    # config 2 (headline) and config 4's shard: HBM bytes per launch against the algorithmic bytes
    if os.path.exists(f"{p}/pmc_fetch_size.csv"):
        pmc_summary.main(p, os.path.join(ROOT, "profiles", "pmc_rollout_bandit.json"),
                         algorithmic=bench.algorithmic_bytes(4096, 500, 4))
    if os.path.exists(f"{p}/linear_pmc_fetch_size.csv"):
        d = os.path.join(p, "_linear")
        os.makedirs(d, exist_ok=True)
        for f in ("pmc_fetch_size.csv", "pmc_write_size.csv", "pmc_tcc_hit_miss.csv"):
            shutil.copy(f"{p}/linear_{f}", f"{d}/{f}")
        pmc_summary.main(d, os.path.join(ROOT, "profiles", "pmc_rollout_linear.json"),
                         algorithmic=bench.algorithmic_bytes(4096, 1000, 4))
        shutil.rmtree(d)
    if os.path.isdir(f"{g}/prof_dr_{tag}/trace"):
        pmc_darkroom.main(f"{g}/prof_dr_{tag}", os.path.join(ROOT, "profiles", "pmc_rollout_darkroom.json"))


if __name__ == "__main__":
    main(sys.argv[1])
