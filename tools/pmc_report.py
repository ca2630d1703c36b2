"""Turn two rocprofv3 --pmc passes (WRITE_SIZE, FETCH_SIZE) into the per-launch
HBM traffic of the roofline kernel, written as JSON under profiles/.

    python tools/pmc_report.py gpurun_out/pmc_WRITE_SIZE gpurun_out/pmc_FETCH_SIZE \
        --kernel "observe_kernel<false>" --out profiles/r01_pmc_observe.json

Units and corrections follow /opt/skills/guides/MI355X_MICROARCH.md (HBM /
rocprofv3 section): both counters are in KiB; WRITE_SIZE is exact for the
16 B/lane streaming stores the observe kernel issues; FETCH_SIZE counts 64 B per
128-B line fetched -- half the bytes of wide (16 B/lane) streaming reads (the
guide) and half the distinct 128-B lines of the kernels' narrow dword reads too
(calibrated in round 5 on the BFS-window pattern: tools/fetch_calib.hip,
profiles/r05_fetch_calibration.json) -- so traffic = WRITE + 2 x FETCH.
"""
import argparse
import csv
import glob
import json
import os


def per_launch(d, counter, kernel):
    files = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    assert files, f"no counter_collection.csv under {d}"
    vals = []
    for f in files:
        for r in csv.DictReader(open(f)):
            if r["Counter_Name"] == counter and kernel in r["Kernel_Name"]:
                vals.append(float(r["Counter_Value"]))
    assert vals, f"{counter}: no dispatch of {kernel}"
    return sum(vals) / len(vals), len(vals)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("write_dir")
    ap.add_argument("fetch_dir")
    ap.add_argument("--kernel", default="observe_kernel<false>")
    ap.add_argument("--algorithmic-bytes", type=float, default=None,
                    help="algorithmic bytes per launch, for the ratio")
    ap.add_argument("--steps-per-launch", type=int, default=1,
                    help="lockstep steps one launch of the kernel runs (mapf_rollout_random: T)")
    ap.add_argument("--out", required=True)
    a = ap.parse_args()
    w_kib, nw = per_launch(a.write_dir, "WRITE_SIZE", a.kernel)
    f_kib, nf = per_launch(a.fetch_dir, "FETCH_SIZE", a.kernel)
    w, f = w_kib * 1024.0, f_kib * 1024.0
    rep = {
        "kernel": a.kernel, "launches": {"WRITE_SIZE": nw, "FETCH_SIZE": nf},
        "write_bytes": w, "fetch_bytes_raw": f, "fetch_bytes_x2": 2 * f,
        "traffic_bytes": w + 2 * f,
        "steps_per_launch": a.steps_per_launch,
        "note": "per launch; counters in KiB x1024; WRITE_SIZE exact for 16 B/lane stores; "
                "FETCH_SIZE = 64 B per 128-B line read (calibrated: profiles/r05_fetch_calibration.json): "
                "traffic = WRITE + 2 x FETCH",
    }
    if a.algorithmic_bytes:
        rep["algorithmic_bytes"] = a.algorithmic_bytes
        rep["traffic_over_algorithmic"] = (w + 2 * f) / a.algorithmic_bytes
    os.makedirs(os.path.dirname(a.out) or ".", exist_ok=True)
    json.dump(rep, open(a.out, "w"), indent=1)
    print(json.dumps(rep))


if __name__ == "__main__":
    main()
