"""Copy a tools/profile.sh run (gpurun_out/<TAG>/) into profiles/<TAG>/ and derive the per-launch
HBM traffic of the sample-mode render kernel from the PMC passes -> an entry of profiles/traffic.json
(read by bench.py for `roofline.traffic`), keyed by workload, spp, RNG mode, kernel and the
build id (sha256 of libpt.so) the run measured: bench.py reports the counters only for that build.

HBM bytes per launch = 2 x FETCH_SIZE + WRITE_SIZE (rocprofv3 reports both in KiB; on gfx950
FETCH_SIZE counts half of the bytes of 128-B requests, MI355X_MICROARCH.md "HBM"), taken from the
wavefront render launch of `bench.py --steps 1 --warmup 0 --no-compat` (warmup launch 1 is the
ray-synchronous kernel, launch 2 the timed wavefront kernel).

    python tools/collect_profile.py r01_final
"""
import csv
import json
import os
import shutil
import statistics
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def render_launches(path, counter):
    rows = [r for r in csv.DictReader(open(path)) if r["Counter_Name"] == counter]
    return [(r["Kernel_Name"], float(r["Counter_Value"])) for r in rows if "renderKernel" in r["Kernel_Name"]]


def main(tag):
    src = os.path.join(REPO, "gpurun_out", tag)
    dst = os.path.join(REPO, "profiles", tag)
    os.makedirs(dst, exist_ok=True)
    shutil.copy(os.path.join(src, "bench.json"), os.path.join(dst, "bench.json"))
    shutil.copy(os.path.join(src, "trace", "run_kernel_stats.csv"), os.path.join(dst, "kernel_stats.csv"))
    with open(os.path.join(src, "trace", "run_kernel_trace.csv")) as f, \
            open(os.path.join(dst, "kernel_trace_render.csv"), "w") as g:
        lines = f.readlines()
        g.write(lines[0])
        g.writelines(l for l in lines[1:] if "render" in l or "resolve" in l)
    for p in ("fetch", "write", "tcc", "sq", "valu"):
        if os.path.exists(os.path.join(src, f"pmc_{p}", "run_counter_collection.csv")):
            shutil.copy(os.path.join(src, f"pmc_{p}", "run_counter_collection.csv"), os.path.join(dst, f"pmc_{p}.csv"))

    bench = json.loads(open(os.path.join(src, "bench.json")).read())
    fetch = render_launches(os.path.join(dst, "pmc_fetch.csv"), "FETCH_SIZE")
    write = render_launches(os.path.join(dst, "pmc_write.csv"), "WRITE_SIZE")
    wf_fetch = [v for k, v in fetch if "renderKernelWF" in k] or [fetch[-1][1]]
    wf_write = [v for k, v in write if "renderKernelWF" in k] or [write[-1][1]]
    # the median launch: a run of several frames holds a cost-measuring launch every few frames
    # (the tile order's refresh: one more atomic per task), the steady-state launches are the rest
    fetch_b = 2.0 * steady(wf_fetch) * 1024.0
    write_b = steady(wf_write) * 1024.0
    cfg = bench["config"]
    out = {
        "workload": cfg["workload"], "spp": cfg["spp"], "rng": cfg["rng"],
        "kernel": "wide" if "WIDE=true" in bench["roofline"].get("kernel", "") else "wavefront",
        "traffic_bytes_per_launch": fetch_b + write_b,
        "fetch_bytes": fetch_b, "write_bytes": write_b,
        "source": f"profiles/{tag}/pmc_fetch.csv + pmc_write.csv (separate rocprofv3 --pmc passes; "
                  "2 x FETCH_SIZE + WRITE_SIZE, KiB -> B; the factor 2 calibrated for this access shape -- "
                  "random 80-B records at an 80-B stride, one 128-B request per line -- in "
                  "profiles/r04_fetch_calib/fetch_calib.json; the counters include Infinity-Cache hits, "
                  "so this is the traffic past L2, an upper bound of the HBM traffic)",
    }
    out["build_id"] = bench["build_id"]
    # TCC (L2) hits and misses of the same launch, when that pass ran: is the tree L2-resident?
    tcc_csv = os.path.join(dst, "pmc_tcc.csv")
    if os.path.exists(tcc_csv):
        hit = [v for k, v in render_launches(tcc_csv, "TCC_HIT_sum") if "renderKernelWF" in k]
        miss = [v for k, v in render_launches(tcc_csv, "TCC_MISS_sum") if "renderKernelWF" in k]
        if hit and miss:
            out["tcc_hit"], out["tcc_miss"] = steady(hit), steady(miss)
            out["tcc_hit_rate"] = out["tcc_hit"] / max(1.0, out["tcc_hit"] + out["tcc_miss"])
    store("traffic", out)
    print(json.dumps(out, indent=1))
    # VALU wave-instructions per launch of the timed (wavefront) render kernel: the wide kernel's
    # binding resource, reported by bench.py as roofline.valu_issue
    valu_csv = os.path.join(dst, "pmc_valu.csv")
    if os.path.exists(valu_csv):
        valu = [v for k, v in render_launches(valu_csv, "SQ_INSTS_VALU") if "renderKernelWF" in k]
        if valu:
            v = {key: out[key] for key in ("workload", "spp", "rng", "kernel")}
            v["valu_wave_instructions_per_launch"] = steady(valu)
            v["source"] = f"profiles/{tag}/pmc_valu.csv (rocprofv3 --pmc SQ_INSTS_VALU, one frame)"
            v["build_id"] = bench["build_id"]
            store("valu", v)
            print(json.dumps(v, indent=1))


def steady(vals):
    """The median of a run's wavefront render launches (the single launch of a one-frame run)."""
    return float(statistics.median(vals))


def store(name, entry):
    """profiles/<name>.json = {"entries": [...]}: one entry per workload (the newest run replaces
    the entry of the same workload, spp, RNG mode and kernel)."""
    path = os.path.join(REPO, "profiles", name + ".json")
    try:
        data = json.load(open(path))
        entries = data.get("entries", [])
    except (OSError, ValueError):
        entries = []
    key = lambda e: (e.get("workload"), e.get("spp"), e.get("rng"), e.get("kernel"))  # noqa: E731
    entries = [e for e in entries if key(e) != key(entry)] + [entry]
    with open(path, "w") as f:
        json.dump({"entries": entries}, f, indent=1)


if __name__ == "__main__":
    main(sys.argv[1])
