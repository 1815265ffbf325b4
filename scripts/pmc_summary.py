"""Summarise a rocprofv3 PMC pass of the headline kernel into profiles/pmc_rollout_bandit.json.

HBM bytes per launch = (2 * FETCH_SIZE + WRITE_SIZE) * 1024:
FETCH_SIZE/WRITE_SIZE are in KiB; on gfx950 FETCH_SIZE reports exactly half the
bytes of a wide (16 B/lane) coalesced streaming read (MI355X_MICROARCH.md §HBM),
which is the access form of the K/V stream (global_load_dwordx4), so it is doubled.
WRITE_SIZE is exact for 16-B-per-lane stores only; the K/V append is 4-B stores,
so the write side is an upper bound.
"""
import csv
import json
import sys


def counter(path, name, kernel):
    vals = [float(r["Counter_Value"]) for r in csv.DictReader(open(path))
            if kernel in r["Kernel_Name"] and r["Counter_Name"] == name]
    return sum(vals) / len(vals)


def main(d, out, kernel="rollout_bandit_kernel", algorithmic=None):
    fetch = counter(f"{d}/pmc_fetch_size.csv", "FETCH_SIZE", kernel)
    write = counter(f"{d}/pmc_write_size.csv", "WRITE_SIZE", kernel)
    hit = counter(f"{d}/pmc_tcc_hit_miss.csv", "TCC_HIT_sum", kernel)
    miss = counter(f"{d}/pmc_tcc_hit_miss.csv", "TCC_MISS_sum", kernel)
    res = {"kernel": kernel, "FETCH_SIZE_KiB": fetch, "WRITE_SIZE_KiB": write,
           "hbm_read_bytes_corrected": 2 * fetch * 1024, "hbm_write_bytes": write * 1024,
           "hbm_bytes_per_launch": (2 * fetch + write) * 1024, "l2_hit_rate": hit / (hit + miss),
           "note": "FETCH_SIZE doubled per gfx950 calibration; WRITE_SIZE uncalibrated for 4-B stores"}
    if algorithmic:
        res["algorithmic_bytes_per_launch"] = algorithmic
        res["traffic_over_algorithmic"] = res["hbm_bytes_per_launch"] / algorithmic
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2], algorithmic=int(sys.argv[3]) if len(sys.argv) > 3 else None)
