"""HBM activity beside the PMC counters (diagnostic): no user-mode profiler counter separates
Infinity-Cache hits from HBM reads on this box (profiles/r05_counters), so this samples the
firmware's memory-controller activity (`amd-smi metric --usage`: UMC_ACTIVITY, %) while a workload
runs: idle, a device-to-device copy of known bandwidth (calibration), and render frames of the
given configurations (sample mode) back to back.

    python tools/hbm_activity.py [seconds per workload] [configs...]   -> JSON lines
"""
import json
import os
import subprocess
import sys
import threading
import time

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "path-tracer-cuda-opengl_amd", "python"))
import ptamd  # noqa: E402

SAMPLES = []
STOP = threading.Event()


def sampler():
    while not STOP.is_set():
        t = time.time()
        try:
            out = subprocess.run(["amd-smi", "metric", "-g", "0", "--usage", "--json"], capture_output=True,
                                 text=True, timeout=10).stdout
            SAMPLES.append((t, time.time(), out))
        except Exception as e:   # noqa: BLE001
            SAMPLES.append((t, time.time(), f"error {e}"))
        time.sleep(0.05)


def umc(text):
    try:
        d = json.loads(text)
    except ValueError:
        return None
    if isinstance(d, dict) and "gpu_data" in d:
        d = d["gpu_data"]
    d = d[0] if isinstance(d, list) else d
    u = d.get("usage", d)
    v = u.get("umc_activity") or u.get("UMC_ACTIVITY")
    if isinstance(v, dict):
        v = v.get("value")
    try:
        return float(v)
    except (TypeError, ValueError):
        return None


def window(t0, t1):
    vals = [umc(o) for a, b, o in SAMPLES if a >= t0 and b <= t1]
    vals = [v for v in vals if v is not None]
    return {"n": len(vals), "mean": sum(vals) / len(vals) if vals else None, "max": max(vals) if vals else None}


def main():
    secs = float(sys.argv[1]) if len(sys.argv) > 1 else 6.0
    cfgs = sys.argv[2:] or ["c5x4", "c5", "c3"]
    th = threading.Thread(target=sampler, daemon=True)
    th.start()
    time.sleep(2.0)
    print(json.dumps({"first_sample": SAMPLES[0][2][:2000] if SAMPLES else None}), flush=True)
    t0 = time.time()
    time.sleep(secs)
    print(json.dumps({"workload": "idle", "umc": window(t0, time.time())}), flush=True)
    # calibration: device-to-device copies of 4 GiB (read + write 8 GiB per copy)
    a = torch.empty(1 << 30, dtype=torch.float32, device="cuda")
    b = torch.empty_like(a)
    torch.cuda.synchronize()
    t0 = time.time()
    n = 0
    while time.time() - t0 < secs:
        b.copy_(a)
        n += 1
        if n % 8 == 0:
            torch.cuda.synchronize()
    torch.cuda.synchronize()
    el = time.time() - t0
    print(json.dumps({"workload": "copy 4 GiB", "tb_per_s": n * 2 * (4 << 30) / el / 1e12,
                      "umc": window(t0 + 0.5, time.time())}), flush=True)
    del a, b
    torch.cuda.empty_cache()
    names = {"c2": "cornell", "c3": "bunny_cornell", "c5": "bunny_field", "c5x4": "bunny_field_x4"}
    for cfg in cfgs:
        p = ptamd.Preset(names[cfg])
        scene = ptamd.Scene(p.objects, p.materials)
        film = ptamd.Film(p.width, p.height, 1)
        spp = {"c3": 256, "c5": 128}.get(cfg, p.spp)
        ptamd.render(scene, film, p.camera, spp, p.max_depth, rng=ptamd.RNG_SAMPLE)   # (tree build, order)
        t0 = time.time()
        n = rays = 0
        kms = 0.0
        while time.time() - t0 < secs:
            _, st = ptamd.render(scene, film, p.camera, spp, p.max_depth, rng=ptamd.RNG_SAMPLE)
            n += 1
            rays += st.rays
            kms += st.kernel_ms
        print(json.dumps({"workload": cfg, "spp": spp, "frames": n, "kernel_ms": kms / n,
                          "mray_s": rays / (kms / 1e3) / 1e6, "umc": window(t0 + 0.5, time.time())}), flush=True)
        del scene, film
    STOP.set()


if __name__ == "__main__":
    main()
