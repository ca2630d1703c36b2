"""Mean per-dispatch value of every counter found under rocprofv3 --pmc output
directories, per kernel (name prefix match), as one table.

    python tools/pmc_table.py gpurun_out/sq_1 gpurun_out/sq_2 --kernel step_observe_kernel
"""
import argparse
import collections
import csv
import glob
import os


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dirs", nargs="+")
    ap.add_argument("--kernel", default="step_observe_kernel")
    a = ap.parse_args()
    acc = collections.defaultdict(list)
    for d in a.dirs:
        for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
            per = collections.defaultdict(float)      # (dispatch, counter) -> summed over dimensions
            for r in csv.DictReader(open(f)):
                if a.kernel in r["Kernel_Name"]:
                    per[(r.get("Dispatch_Id", ""), r["Counter_Name"])] += float(r["Counter_Value"])
            for (_, c), v in per.items():
                acc[(os.path.basename(d.rstrip("/")), c)].append(v)
    for (d, c), v in sorted(acc.items()):
        print(f"{d:14s} {c:24s} {sum(v) / len(v):16.1f}   ({len(v)} dispatches)")


if __name__ == "__main__":
    main()
