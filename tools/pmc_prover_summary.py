"""Per-kernel PMC summary of the prover (tools/gpu_pmc_prover.sh output) ->
profiles/<tag>_pmc_prover.json.

Per kernel (mean over launches of the batch-size shape that dominates):
VGPRs, waves, VALU instructions per wave, busy / wave cycles, the fraction of
wave cycles issuing VALU (SQ_ACTIVE_INST_VALU / SQ_WAVE_CYCLES, both
quad-cycle counters), waves resident per SIMD (SQ_WAVE_CYCLES /
SQ_BUSY_CYCLES / 1024 SIMDs... see `waves_per_simd`), the effective clock
(GRBM_GUI_ACTIVE / 8 XCDs / duration) and HBM-side bytes (2 x FETCH_SIZE +
WRITE_SIZE, MI355X_MICROARCH.md gfx950 correction).

    python tools/pmc_prover_summary.py gpurun_out/pmc_prover_r02a r02a
"""
import collections
import csv
import json
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
KERNELS = ("k_ipa_round_dt", "k_dt_msm", "k_pedersen", "k_ipa_fold", "k_ipa_terms", "k_ipa_cross_final", "k_poly_coef", "k_poly_x",
           "k_verify_replay_g", "k_verify_replay_post", "k_verify_consts", "k_verify_decompress",
           "k_compress_p3", "k_decompress", "k_msm_accumulate", "k_msm_reduce_wave", "k_sc_halve", "k_verify_scalars")


def load(path):
    # (kernel, dispatch) -> {counter: value}, plus per-dispatch meta
    disp = collections.defaultdict(dict)
    meta = {}
    for r in csv.DictReader(open(path)):
        name = r["Kernel_Name"].split("(")[0].replace("void ", "").split("<")[0]
        key = (name, int(r["Dispatch_Id"]))
        disp[key][r["Counter_Name"]] = float(r["Counter_Value"])
        meta[key] = {"grid": int(r["Grid_Size"]), "wg": int(r["Workgroup_Size"]), "vgpr": int(r["VGPR_Count"]),
                     "lds": int(r["LDS_Block_Size"]),
                     "ns": int(r["End_Timestamp"]) - int(r["Start_Timestamp"])}
    return disp, meta


def main():
    src, tag = Path(sys.argv[1]), sys.argv[2]
    merged = collections.defaultdict(dict)
    meta = {}
    for p in sorted(src.glob("p*/run_counter_collection.csv")):
        d, m = load(p)
        for k, v in d.items():
            # dispatch ids are per run: key by (kernel, launch ordinal) instead
            merged[(p.parent.name,) + k].update(v)
        meta.update({(p.parent.name,) + k: v for k, v in m.items()})
    out = {}
    for kern in KERNELS:
        rows = collections.defaultdict(list)  # counter -> values over launches (all passes)
        grids = collections.Counter()
        for key, cnt in merged.items():
            if key[1] != kern:
                continue
            grids[meta[key]["grid"]] += 1
        if not grids:
            continue
        grid = grids.most_common(1)[0][0]  # the dominant launch shape
        m0 = None
        for key, cnt in merged.items():
            if key[1] != kern or meta[key]["grid"] != grid:
                continue
            m0 = meta[key]
            for c, v in cnt.items():
                rows[c].append(v)
            rows["_ns"].append(meta[key]["ns"])
        mean = {c: sum(v) / len(v) for c, v in rows.items()}
        e = {"grid_threads": grid, "workgroup": m0["wg"], "vgprs": m0["vgpr"], "lds_bytes": m0["lds"],
             "launches_sampled": len(rows["_ns"]), "duration_us_profiled": mean["_ns"] / 1e3}
        if "SQ_WAVES" in mean:
            w = mean["SQ_WAVES"]
            e["waves"] = w
            e["valu_insts_per_wave"] = mean["SQ_INSTS_VALU"] / w
            e["valu_issue_frac"] = mean["SQ_ACTIVE_INST_VALU"] / mean["SQ_WAVE_CYCLES"]
            e["any_issue_frac"] = mean["SQ_ACTIVE_INST_ANY"] / mean["SQ_WAVE_CYCLES"]
            e["wait_any_frac"] = mean["SQ_WAIT_ANY"] / mean["SQ_WAVE_CYCLES"]
            e["wait_inst_any_frac"] = mean["SQ_WAIT_INST_ANY"] / mean["SQ_WAVE_CYCLES"]
            e["eff_clock_ghz"] = mean["GRBM_GUI_ACTIVE"] / 8 / mean["_ns"] if mean["_ns"] > 0 else None
            # mean resident waves per SIMD over the launch: SQ_WAVE_CYCLES is
            # the sum over waves of their resident time in quad-cycles
            # (MI355X_MICROARCH.md: SQ_WAVE_CYCLES counts quad-cycles), the
            # launch spans GRBM_GUI_ACTIVE / 8 XCDs cycles, on 1024 SIMDs.
            # Check (round 3's WAVE/BUSY/32 read 0.48 for the accumulate): a
            # launch of more waves than fit reads at most its occupancy --
            # k_verify_decompress (244 VGPRs, 2 waves per SIMD, 7.9 launched
            # per SIMD) reads 1.78; the 2^20 accumulate (4100 waves) reads
            # 1.77 in the bench stream, where it carries the 13 KB LDS pad
            # beside another MSM (3 workgroups per CU: its 1025 workgroups
            # take 1.33 rounds, ~2 waves per SIMD averaged over the launch),
            # and config 5's lone one (961 workgroups) 2.24 although 4 of its
            # 40 KB workgroups fit a CU (tools/ubench/lds_occ.hip: 3.9
            # resident at 40960 B, 3.0 at 41216) -- a launch-average that
            # also counts the tail, read it relative.  (rocprofv3's
            # VGPR_Count column reads half the compiler's count on gfx950.)
            cyc = mean["GRBM_GUI_ACTIVE"] / 8
            e["waves_per_simd"] = 4.0 * mean["SQ_WAVE_CYCLES"] / max(cyc, 1) / 1024
            e["launch_waves_per_simd"] = w / 1024
            for c in ("SQ_WAVE_CYCLES", "SQ_BUSY_CYCLES", "GRBM_GUI_ACTIVE"):
                e[c.lower()] = mean[c]
        for c in ("SQ_INSTS_SALU", "SQ_INSTS_VMEM_RD", "SQ_INSTS_VMEM_WR", "SQ_INSTS_LDS", "SQ_LDS_BANK_CONFLICT",
                  "SQ_INSTS_BRANCH"):
            if c in mean and "SQ_WAVES" in mean:
                e[c.lower() + "_per_wave"] = mean[c] / mean["SQ_WAVES"]
        if "FETCH_SIZE" in mean and "WRITE_SIZE" in mean:
            e["hbm_bytes"] = 2 * mean["FETCH_SIZE"] * 1024 + mean["WRITE_SIZE"] * 1024
        out[kern] = e
    dst = ROOT / "profiles" / f"{tag}_pmc_prover.json"
    dst.write_text(json.dumps(out, indent=1) + "\n")
    for k, e in out.items():
        print(k, {a: (round(b, 3) if isinstance(b, float) else b) for a, b in e.items()})


if __name__ == "__main__":
    main()
