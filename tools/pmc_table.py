"""Per-kernel sums of every counter in one or more rocprofv3 --pmc counter_collection.csv files.

    python tools/pmc_table.py DIR [DIR ...] [--div N] [--filter REGEX]

Values are summed over dispatches and divided by --div (frames rendered in the run, default 2:
tools/tune_wavefront.py renders a warm-up frame and a timed one).  FETCH_SIZE is doubled
(gfx950's half-count of 16-B/lane reads, MI355X_MICROARCH.md § HBM) and shown in GB like
WRITE_SIZE; the other counters are raw counts (1e6)."""
import collections
import csv
import os
import re
import sys


def short(name):
    name = re.sub(r"\(anonymous namespace\)::", "", name)
    name = re.sub(r"^void ", "", name)
    return re.sub(r"\(.*$", "", name)


def main():
    args, div, filt = [], 2.0, None
    it = iter(sys.argv[1:])
    for a in it:
        if a == "--div":
            div = float(next(it))
        elif a == "--filter":
            filt = re.compile(next(it))
        else:
            args.append(a)
    tot = collections.defaultdict(lambda: collections.defaultdict(float))
    disp = collections.defaultdict(set)
    counters = []
    for d in args:
        f = os.path.join(d, "run_counter_collection.csv")
        for row in csv.DictReader(open(f)):
            k = short(row["Kernel_Name"])
            if filt and not filt.search(k):
                continue
            c = row["Counter_Name"]
            if c not in counters:
                counters.append(c)
            v = float(row["Counter_Value"])
            if c == "FETCH_SIZE":
                v *= 2
            tot[k][c] += v
            disp[(k, c)].add(row["Dispatch_Id"])
    print("| kernel | " + " | ".join(counters) + " |")
    print("|---|" + "---:|" * len(counters))
    for k in sorted(tot, key=lambda k: -max(tot[k].values())):
        cells = []
        for c in counters:
            v = tot[k].get(c, 0.0) / div
            cells.append(f"{v / 1e6:.3f} GB" if c in ("FETCH_SIZE", "WRITE_SIZE") else f"{v / 1e6:.2f} M")
        print(f"| {k} | " + " | ".join(cells) + " |")


if __name__ == "__main__":
    main()
