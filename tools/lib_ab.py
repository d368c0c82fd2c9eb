"""Interleaved A/B of library builds (GPU): tools/one_frame.py per build, PT_LIB selecting it.

    python tools/lib_ab.py c3 256 3 base:path-tracer-cuda-opengl_amd/libpt.so x:variants/libpt_x.so[:chunk]

Each round runs every build once (a fresh process: REPEAT=2 frames, the faster kept), so clock
drift hits all builds alike; prints the median kernel ms per build and each build's image digest.
"""
import json
import os
import statistics
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main():
    cfg, spp, rounds = sys.argv[1], sys.argv[2], int(sys.argv[3])
    libs = []   # name:lib[:chunk[:ENV=V,ENV=V]]
    for v in sys.argv[4:]:
        parts = v.split(":")
        libs.append((parts[0], parts[1], parts[2] if len(parts) > 2 else "0", parts[3] if len(parts) > 3 else ""))
    times = {n: [] for n, _, _, _ in libs}
    digests = {}
    work = {}
    for r in range(rounds):
        for name, lib, chunk, envs in libs:
            env = dict(os.environ, PT_LIB=os.path.join(REPO, lib), REPEAT=os.environ.get("REPEAT", "2"))
            env.update(dict(e.split("=", 1) for e in envs.split(",") if e))
            out = subprocess.run([sys.executable, os.path.join(REPO, "tools", "one_frame.py"), cfg, spp, os.environ.get("RNG", "sample"), chunk],
                                 env=env, capture_output=True, text=True, timeout=300)
            if out.returncode != 0:
                print(name, "failed", out.stderr[-800:], flush=True)
                sys.exit(1)
            d = json.loads(out.stdout.strip().splitlines()[-1])
            times[name].append(d["kernel_ms"])
            digests[name] = d["image"]
            work[name] = {"node_visits": d.get("node_visits"), "tri_tests": d.get("tri_tests")}
            print(f"round {r} {name}: {d['kernel_ms']:.2f} ms", flush=True)
    for name, _, _, _ in libs:
        print(json.dumps({"build": name, "median_ms": statistics.median(times[name]), "all": times[name],
                          "image": digests[name], **work[name]}))


if __name__ == "__main__":
    main()
