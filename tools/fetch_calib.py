"""Summarise a tools/fetch_calib.sh run (gpurun_out/fetch_calib/) into profiles/<tag>/fetch_calib.json
and copy its counter CSVs there.

For each access mode of tools/micro/fetch_calib.hip: the bytes the lanes requested, the 128-B lines
and 64-B sectors they cover (known by construction), and per counter the value of the measured
launch (the last gather launch of the run).  Derived: FETCH_SIZE bytes / line bytes (the factor
that turns FETCH_SIZE into past-L2 line traffic for that access shape), requests per line.

    python tools/fetch_calib.py r04_fetch_calib
"""
import csv
import json
import os
import shutil
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(REPO, "gpurun_out", "fetch_calib")


def last_launch(path):
    """counter -> value summed over the instances / XCDs of the last non-fill dispatch"""
    rows = [r for r in csv.DictReader(open(path)) if "fillBuffer" not in r["Kernel_Name"]]
    last = max(int(r["Dispatch_Id"]) for r in rows)
    out = {}
    for r in rows:
        if int(r["Dispatch_Id"]) == last:
            out[r["Counter_Name"]] = out.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    return out


def main(tag):
    dst = os.path.join(REPO, "profiles", tag)
    os.makedirs(dst, exist_ok=True)
    modes = []
    for mode in ("stream", "g128", "g64s128", "g80s128", "g80", "g80mall", "g80warm", "g48"):
        jpath = os.path.join(SRC, mode + ".json")
        if not os.path.exists(jpath):
            continue
        m = json.loads(open(jpath).read().strip().splitlines()[-1])
        ctr = {}
        for p in ("fetch", "ea", "hit", "bub"):
            c = os.path.join(SRC, f"{mode}_{p}", "run_counter_collection.csv")
            if os.path.exists(c):
                ctr.update(last_launch(c))
                shutil.copy(c, os.path.join(dst, f"{mode}_{p}.csv"))
        line_bytes = m["lines128"] * 128
        if "FETCH_SIZE" in ctr:
            m["fetch_size_bytes"] = ctr["FETCH_SIZE"] * 1024
            m["fetch_size_over_line_bytes"] = m["fetch_size_bytes"] / line_bytes
            m["fetch_size_over_requested_bytes"] = m["fetch_size_bytes"] / m["requested_bytes"]
        if "TCC_EA0_RDREQ_sum" in ctr:
            m["rdreq_per_line"] = ctr["TCC_EA0_RDREQ_sum"] / m["lines128"]
        m["line_bytes_per_s"] = line_bytes / (m["ms"] * 1e-3)
        m["counters"] = ctr
        modes.append(m)
    out = {"tool": "tools/micro/fetch_calib.hip via tools/fetch_calib.sh (separate rocprofv3 --pmc passes)",
           "modes": modes}
    with open(os.path.join(dst, "fetch_calib.json"), "w") as f:
        json.dump(out, f, indent=1)
    for m in modes:
        print(f"{m['mode']:8s} req/line {m.get('rdreq_per_line', float('nan')):.3f}  FETCH/line-bytes "
              f"{m.get('fetch_size_over_line_bytes', float('nan')):.3f}  FETCH/requested "
              f"{m.get('fetch_size_over_requested_bytes', float('nan')):.3f}  "
              f"bubble {m['counters'].get('TCC_BUBBLE_sum', float('nan')):.0f}  dram {m['counters'].get('TCC_EA0_RDREQ_DRAM_sum', float('nan')):.0f}  "
              f"{m['ms']:.3f} ms  {m['line_bytes_per_s'] / 1e12:.2f} TB/s of lines")


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "r04_fetch_calib")
