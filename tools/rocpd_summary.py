"""Per-kernel summary of a rocprofv3 database (--kernel-trace, default rocpd output): name, calls,
total / average / min duration, grid, VGPRs -- and, with --per <substring>, the totals divided by
the call count of the kernel matching <substring> (e.g. one acting forward or one rollout step).
  python3 tools/rocpd_summary.py gpurun_out/<dir>/<name>_results.db --per conv_first_kernel"""
import argparse
import collections
import sqlite3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--per", default=None)
    ap.add_argument("--top", type=int, default=40)
    args = ap.parse_args()
    c = sqlite3.connect(args.db)
    agg = collections.OrderedDict()
    for name, dur, gx, wx, vg, ag in c.execute(
            "select name, duration, grid_x, workgroup_x, vgpr_count, accum_vgpr_count from kernels"):
        a = agg.setdefault(name, {"calls": 0, "total": 0, "min": None, "grid": gx // max(wx, 1), "vgpr": vg + ag})
        a["calls"] += 1
        a["total"] += dur
        a["min"] = dur if a["min"] is None else min(a["min"], dur)
    per = None
    if args.per:
        hits = [a["calls"] for n, a in agg.items() if args.per in n]
        per = max(hits) if hits else None
    tot = sum(a["total"] for a in agg.values())
    hdr = f"{'us/unit' if per else 'total_us':>10} {'share':>6} {'calls':>7} {'avg_us':>9} {'min_us':>9} {'wgs':>7} {'regs':>5}  kernel"
    print(f"# {args.db}: {sum(a['calls'] for a in agg.values())} dispatches, {tot / 1e3:.1f} us total"
          + (f"; per unit = per call of '{args.per}' ({per} calls): {tot / 1e3 / per:.1f} us" if per else ""))
    print(hdr)
    for n, a in sorted(agg.items(), key=lambda kv: -kv[1]["total"])[:args.top]:
        v = a["total"] / 1e3 / (per or 1)
        print(f"{v:10.1f} {a['total'] / tot:6.3f} {a['calls']:7d} {a['total'] / a['calls'] / 1e3:9.1f} "
              f"{a['min'] / 1e3:9.1f} {a['grid']:7d} {a['vgpr']:5d}  {n[:110]}")


if __name__ == "__main__":
    main()
