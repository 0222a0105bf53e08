"""Per-kernel means of the MFMA / busy counters collected by
tools/pmc_mfma.sh (rocprofv3 counter_collection CSVs), for the kernels of the
GMRES Arnoldi step and block CG."""
import csv
import json
import os
import sys
from collections import defaultdict


def main(out):
    res = {}
    for prog in ("gmres_metric", "cfg4"):
        path = os.path.join(out, prog, "run_counter_collection.csv")
        acc = defaultdict(lambda: defaultdict(list))
        with open(path) as f:
            for row in csv.DictReader(f):
                name = row["Kernel_Name"].split("(")[0].replace("void ", "")
                acc[name][row["Counter_Name"]].append(float(row["Counter_Value"]))
        res[prog] = {k: {c: sum(v) / len(v) for c, v in cs.items()} | {"dispatches": max(len(v) for v in cs.values())}
                     for k, cs in acc.items()}
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main(sys.argv[1])
