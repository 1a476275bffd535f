"""Timeline of the last config-5 batch verification in a rocprofv3
kernel + memory-copy trace (tools/verify_stages.py under
`rocprofv3 --kernel-trace --memory-copy-trace`): every kernel and copy from
the end of the previous verification, in us from its first event.

    python tools/verify_timeline.py gpurun_out/vtl
"""
import csv
import sys
from pathlib import Path


def main():
    d = Path(sys.argv[1])
    ev = []
    for r in csv.DictReader(open(d / "run_kernel_trace.csv")):
        ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), "kernel q%s %s" % (r.get("Queue_Id", "?"),
                                                                                        r["Kernel_Name"].split("(")[0])))
    for r in csv.DictReader(open(d / "run_memory_copy_trace.csv")):
        ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), "copy " + r.get("Direction", "?")))
    ev.sort()
    last = max(i for i, e in enumerate(ev) if "k_verify_replay_g" in e[2])
    j = last
    while j > 0 and "reduce_bits" not in ev[j][2]:
        j -= 1
    t0 = ev[j + 1][0]
    print("start_us  end_us  dur_us  event")
    for e in ev[j + 1:]:
        print("%8.1f %8.1f %7.1f  %s" % ((e[0] - t0) / 1e3, (e[1] - t0) / 1e3, (e[1] - e[0]) / 1e3, e[2]))
        if "reduce_bits" in e[2]:
            break


if __name__ == "__main__":
    main()
