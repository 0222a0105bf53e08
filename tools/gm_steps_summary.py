"""Summarise a rocprofv3 kernel-trace CSV of tools/gm_steps.py: per Arnoldi
step j, the mean duration of the MGS launch (and of the SpMV launch) over the
timed cycles, and a least-squares fit t_mgs(j) = a + b (j + 1).

    python3 tools/gm_steps_summary.py OUT/.../gm_kernel_trace.csv [cycles]
"""
import csv
import sys

import numpy as np


def main(path, cycles=2):
    rows = list(csv.DictReader(open(path)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    mgs = [r for r in rows if "gm_mgs" in r["Kernel_Name"]]
    spmv = [r for r in rows if "spmv" in r["Kernel_Name"]]
    dur = lambda r: (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3  # us
    m = np.array([dur(r) for r in mgs])
    # the last `cycles` cycles of 30 steps each
    m = m[-30 * cycles:].reshape(cycles, 30).mean(axis=0)
    print("kernel", mgs[-1]["Kernel_Name"][:90])
    for j in range(30):
        print(f"j={j:2d}  mgs {m[j]:8.1f} us  per pass {m[j] / (j + 2):6.2f} us")
    x = np.arange(30) + 1.0
    b, a = np.polyfit(x, m, 1)
    print(f"fit: t = {a:.1f} + {b:.2f} * (j + 1) us; mean {m.mean():.1f} us")
    if spmv:
        s = np.array([dur(r) for r in spmv[-30 * cycles:]])
        print(f"spmv mean {s.mean():.1f} us ({spmv[-1]['Kernel_Name'][:60]})")
    # every kernel of the trace, per cycle: tools/gm_steps.py runs one warm-up
    # cycle before the timed ones, so the trace holds cycles + 1 of them
    other = {}
    for r in rows:
        other.setdefault(r["Kernel_Name"][:50], []).append(dur(r))
    for k, v in sorted(other.items(), key=lambda kv: -sum(kv[1]))[:10]:
        print(f"{sum(v) / (cycles + 1) / 1e3:8.3f} ms/cycle  {len(v):5d} calls  {k}")


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 2)
