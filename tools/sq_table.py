"""Per-kernel SQ counter table from rocprofv3 --pmc csv directories (tools/gemm_sq.sh): averages per
dispatch, MFMA utilisation = SQ_VALU_MFMA_BUSY_CYCLES / (1024 SIMDs x GRBM_GUI_ACTIVE / 8), the
effective clock GRBM_GUI_ACTIVE / 8 / duration, and the SQ_WAIT_ANY / SQ_WAVE_CYCLES share."""
import csv
import glob
import os
import sys
from collections import defaultdict


def main(dirs, match):
    acc = defaultdict(lambda: defaultdict(list))
    dur = defaultdict(list)
    for d in dirs:
        for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
            for r in csv.DictReader(open(f)):
                k = r["Kernel_Name"]
                if not any(m in k for m in match):
                    continue
                acc[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
                dur[(k, r["Dispatch_Id"])] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9
    for k, cs in sorted(acc.items()):
        avg = {c: sum(v) / len(v) for c, v in cs.items()}
        ds = [v for (kk, _), v in dur.items() if kk == k]
        t = sum(ds) / len(ds) if ds else float("nan")
        print(k[:110])
        for c in sorted(avg):
            print(f"   {c:28s} {avg[c]:16.0f}")
        g = avg.get("GRBM_GUI_ACTIVE")
        if g:
            print(f"   effective clock {g / 8 / t / 1e9:.2f} GHz over {t * 1e6:.1f} us")
            if "SQ_VALU_MFMA_BUSY_CYCLES" in avg:
                print(f"   MFMA busy {avg['SQ_VALU_MFMA_BUSY_CYCLES'] / (1024 * g / 8):.3f} of the SIMD-cycles")
        if "SQ_WAVE_CYCLES" in avg and "SQ_WAIT_ANY" in avg:
            print(f"   SQ_WAIT_ANY / SQ_WAVE_CYCLES {avg['SQ_WAIT_ANY'] / avg['SQ_WAVE_CYCLES']:.3f}; "
                  f"SQ_WAIT_INST_ANY {avg.get('SQ_WAIT_INST_ANY', 0) / avg['SQ_WAVE_CYCLES']:.3f}; "
                  f"SQ_ACTIVE_INST_ANY {avg.get('SQ_ACTIVE_INST_ANY', 0) / avg['SQ_WAVE_CYCLES']:.3f}")
        if "SQ_LDS_IDX_ACTIVE" in avg and avg["SQ_LDS_IDX_ACTIVE"]:
            print(f"   LDS bank conflict / LDS active {avg.get('SQ_LDS_BANK_CONFLICT', 0) / avg['SQ_LDS_IDX_ACTIVE']:.3f}")


if __name__ == "__main__":
    args = sys.argv[1:]
    i = args.index("--match")
    main(args[:i], args[i + 1:])
