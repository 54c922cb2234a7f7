"""Summarise rocprofv3 --pmc CSVs: per dispatch of the named kernel, counter values (summed over
instances), plus the dispatch duration from the kernel trace.  Usage:
    python tools/pmc_summary.py gpurun_out/pmc [kernel-substring]
"""
import collections
import csv
import json
import pathlib
import sys


def load(dirpath: pathlib.Path, kname: str):
    disp = collections.defaultdict(lambda: collections.defaultdict(float))
    names = {}
    for f in sorted(dirpath.glob("**/run_counter_collection.csv")):
        with open(f) as fh:
            for row in csv.DictReader(fh):
                if kname not in row["Kernel_Name"]:
                    continue
                key = (str(f.parent), int(row["Dispatch_Id"]))
                disp[key][row["Counter_Name"]] += float(row["Counter_Value"])
                names[key] = row["Kernel_Name"]
        tr = f.parent / "run_kernel_trace.csv"
        if tr.exists():
            with open(tr) as fh:
                for row in csv.DictReader(fh):
                    key = (str(f.parent), int(row["Dispatch_Id"]))
                    if key in disp:
                        disp[key]["DURATION_NS"] = float(row["End_Timestamp"]) - float(row["Start_Timestamp"])
    return disp, names


def main():
    d = pathlib.Path(sys.argv[1])
    kname = sys.argv[2] if len(sys.argv) > 2 else "trace_kernel"
    disp, names = load(d, kname)
    # keep, per pass directory, the timed run: the LAST dispatch at least half as long as the longest
    # (the bench's warm-up launch comes first: it rebuilds the cost order and runs without issue
    # priority, so it is not the launch the bench times)
    longest = collections.defaultdict(float)
    for (p, i), c in disp.items():
        longest[p] = max(longest[p], c.get("DURATION_NS", 0))
    best = {}
    for (p, i), c in sorted(disp.items()):
        if c.get("DURATION_NS", 0) >= 0.5 * longest[p]:
            best[p] = (i, c)
    merged = {}
    for p, (i, c) in sorted(best.items()):
        for k, v in c.items():
            if k == "DURATION_NS":
                merged.setdefault("DURATION_NS_" + pathlib.Path(p).name, v)
            else:
                merged[k] = v
    print(json.dumps(merged, indent=1, sort_keys=True))


if __name__ == "__main__":
    main()
