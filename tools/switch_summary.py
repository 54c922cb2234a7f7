"""Per-dispatch table of a `rocprofv3 --pmc ... --kernel-trace` run of tools/switch_probe.py: every
trace_kernel dispatch in launch order with its duration, engine clock (GRBM_GUI_ACTIVE cycles of the
dispatch / its duration; GRBM counts once per XCD on gfx950, so the sum is divided by the 8 XCDs)
and the other counters, joined with the probe's own JSON lines (variant, order state).
    python tools/switch_summary.py <rocprof dir> <probe stdout log>
"""
import collections
import csv
import json
import pathlib
import sys

XCDS = 8


def main():
    d = pathlib.Path(sys.argv[1])
    disp = collections.defaultdict(lambda: collections.defaultdict(float))
    dur = {}
    for f in sorted(d.glob("**/run_counter_collection.csv")):
        with open(f) as fh:
            for row in csv.DictReader(fh):
                if "trace_kernel" not in row["Kernel_Name"]:
                    continue
                disp[int(row["Dispatch_Id"])][row["Counter_Name"]] += float(row["Counter_Value"])
        tr = f.parent / "run_kernel_trace.csv"
        if tr.exists():
            with open(tr) as fh:
                for row in csv.DictReader(fh):
                    dur[int(row["Dispatch_Id"])] = float(row["End_Timestamp"]) - float(row["Start_Timestamp"])
    probe = []
    if len(sys.argv) > 2:
        for line in open(sys.argv[2]):
            line = line.strip()
            if line.startswith("{") and '"i"' in line and '"launches"' not in line:
                probe.append(json.loads(line))
    # the probe's launches are the long dispatches, in order, after the warm-up
    ids = sorted(i for i in disp if dur.get(i, 0) > 0)
    longest = max(dur[i] for i in ids)
    long_ids = [i for i in ids if dur[i] >= 0.3 * longest]
    rows = []
    for k, i in enumerate(long_ids):
        c = disp[i]
        r = {"dispatch": i, "ms": round(dur[i] / 1e6, 2)}
        if "GRBM_GUI_ACTIVE" in c:
            r["clock_GHz"] = round(c["GRBM_GUI_ACTIVE"] / XCDS / dur[i], 3)
        for name in ("SQ_INSTS_VALU", "SQ_WAVES", "SQ_BUSY_CYCLES", "SQ_WAVE_CYCLES"):
            if name in c:
                r[name] = c[name]
        p = k - (len(long_ids) - len(probe))            # the warm-up launch precedes the probe's
        if 0 <= p < len(probe):
            r.update({kk: probe[p][kk] for kk in ("variant", "after", "max_tile_Mcyc", "order_rank_rho")
                      if kk in probe[p]} | {"probe_ms": probe[p]["ms"]})
        rows.append(r)
    for r in rows:
        print(json.dumps(r))


if __name__ == "__main__":
    main()
