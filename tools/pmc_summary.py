"""Summarise a tools/gpu_profile_round.sh output directory into
profiles/pmc_summary.json (per-kernel HBM-side bytes per launch) and
profiles/<tag>_kernel_stats.csv.

FETCH_SIZE / WRITE_SIZE are reported by rocprofv3 in KiB.  Correction per
MI355X_MICROARCH.md §HBM: on gfx950 FETCH_SIZE tallies each 128-B memory
request as 64 B, so bytes read = 2 x FETCH_SIZE.  Verified here on a known
byte count: tools/ubench/gather_cal k_stream (268,435,456 B read -> 131,084
KiB = exactly 1/2).  WRITE_SIZE is taken as exact (the guide's calibration;
k_from_uniform here writes 2^20 x 96 B = 98,304 KiB, matched exactly).

    python tools/pmc_summary.py gpurun_out/prof_r01c r01 20 [proof batch, 384]
"""
import collections
import csv
import json
import shutil
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent


def per_kernel(path):
    d = collections.defaultdict(list)
    for r in csv.DictReader(open(path)):
        d[r["Kernel_Name"].split("(")[0].replace("void ", "").split("<")[0]].append(float(r["Counter_Value"]))
    return d


def main():
    src, tag, log2n = Path(sys.argv[1]), sys.argv[2], int(sys.argv[3])
    batch = int(sys.argv[4]) if len(sys.argv) > 4 else 384  # prove_batch_once.py size (PROOF_BATCH)
    fetch = per_kernel(src / "pmc_fetch" / "run_counter_collection.csv")
    write = per_kernel(src / "pmc_write" / "run_counter_collection.csv")
    out_p = ROOT / "profiles" / "pmc_summary.json"
    out = {}  # regenerated from this run only
    stage_of = {"k_msm_accumulate": "msm_accumulate", "k_rsort_scatter": "msm_scatter_coarse",
                "k_rsort_fine": "msm_scatter_fine", "k_rsort_count": "msm_count", "k_msm_digits": "msm_digits",
                "k_msm_reduce_partial": "msm_reduce", "k_msm_reduce_final": "msm_reduce_final",
                "k_msm_reduce_wave": "msm_reduce_wave", "k_msm_reduce_bits": "msm_reduce_bits",
                "k_msm_fixup_heavy": "msm_fixup", "k_msm_fixup": "msm_fixup", "k_msm_scatter_lds": "msm_scatter_lds", "k_msm_count_lds": "msm_count_lds"}
    for k, st in stage_of.items():
        if k not in fetch or k not in write:
            continue
        # the 2^log2n MSM launches are the most frequent size in the bench run
        f = sum(fetch[k]) / len(fetch[k]) * 1024
        w = sum(write[k]) / len(write[k]) * 1024
        out[f"{st}@2^{log2n}"] = {
            "kernel": k, "launches": len(fetch[k]), "fetch_size_raw_bytes": f, "write_size_bytes": w,
            "read_bytes_corrected": 2 * f, "hbm_bytes_per_launch": 2 * f + w,
            "correction": "read = 2 x FETCH_SIZE (gfx950 128-B requests tallied at 64 B); write exact",
            "source": f"{src.name} ({tag})",
        }
    out_p.write_text(json.dumps(out, indent=1, sort_keys=True) + "\n")
    stats = src / "trace" / "run_kernel_stats.csv"
    if stats.exists():
        shutil.copy(stats, ROOT / "profiles" / f"{tag}_kernel_stats.csv")
    stats = src / "trace_proofs" / "run_kernel_stats.csv"
    if stats.exists():
        shutil.copy(stats, ROOT / "profiles" / f"{tag}_prove_batch{batch}_kernel_stats.csv")
    stats = src / "trace_verify" / "run_kernel_stats.csv"
    if stats.exists():
        shutil.copy(stats, ROOT / "profiles" / f"{tag}_verify4096_kernel_stats.csv")
    b = src / "bench.json"
    if b.exists():
        shutil.copy(b, ROOT / "profiles" / f"{tag}_bench.json")
    print(json.dumps({k: v["hbm_bytes_per_launch"] for k, v in out.items()}, indent=1))


if __name__ == "__main__":
    main()
