"""Per-kernel translation / latency counters from tools/gpu_tlb_prover.sh:
    python tools/tlb_summary.py gpurun_out/tlb_<tag> > profiles/<tag>_tlb_prover.json
Per configuration and kernel (k_dt_msm, k_ipa_round_dt; mean per launch
over the launches of the dominant grid): UTCL1 requests, translation misses
and hits, the miss rate, pending-stall cycles, the mean L2 read latency
(TCP_TCC_READ_REQ_LATENCY / TCP_TCC_READ_REQ, cycles), VALU issue
(SQ_ACTIVE_INST_VALU / SQ_WAVE_CYCLES), wait_any and the UTCL2 busy share."""
import collections
import csv
import json
import sys
from pathlib import Path

KERNELS = ("k_dt_msm", "k_ipa_round_dt")


def rows(d: Path):
    for f in d.rglob("*counter_collection.csv"):
        yield from csv.DictReader(open(f))


def main():
    base = Path(sys.argv[1])
    out = {}
    for c in sorted(base.glob("c*")):
        cfg = (c / "cfg.txt").read_text().strip()
        per = collections.defaultdict(lambda: collections.defaultdict(list))
        grids = collections.defaultdict(collections.Counter)
        for r in rows(c):
            name = r["Kernel_Name"].split("(")[0].replace("void ", "").split("<")[0]
            if name not in KERNELS:
                continue
            grids[name][int(r["Grid_Size"])] += 1
            per[(name, int(r["Grid_Size"]))][r["Counter_Name"]].append(float(r["Counter_Value"]))
        res = {}
        for k in KERNELS:
            if not grids[k]:
                continue
            g = grids[k].most_common(1)[0][0]
            m = {n: sum(v) / len(v) for n, v in per[(k, g)].items()}
            req = m.get("TCP_UTCL1_REQUEST_sum")
            miss = m.get("TCP_UTCL1_TRANSLATION_MISS_sum")
            lat = m.get("TCP_TCC_READ_REQ_LATENCY_sum")
            nreq = m.get("TCP_TCC_READ_REQ_sum")
            wc = m.get("SQ_WAVE_CYCLES")
            res[k] = {"grid": g, "counters": m,
                      "utcl1_miss_rate": miss / req if req and miss is not None else None,
                      "l2_read_latency_cycles": lat / nreq if lat and nreq else None,
                      "valu_issue": m["SQ_ACTIVE_INST_VALU"] / wc if wc and "SQ_ACTIVE_INST_VALU" in m else None,
                      "wait_any": m["SQ_WAIT_ANY"] / wc if wc and "SQ_WAIT_ANY" in m else None,
                      "utcl2_busy": m["GRBM_UTCL2_BUSY"] / m["GRBM_GUI_ACTIVE"]
                      if m.get("GRBM_GUI_ACTIVE") and "GRBM_UTCL2_BUSY" in m else None}
        out[cfg] = res
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
