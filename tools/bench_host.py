"""Host plumbing timing (BASELINE.json config C1 and the (f) "parallel host BVH" row): JSON parse
+ transforms and SAH BVH build of the scene files, sequential vs multi-threaded build (identical
layout, checked).  Runs on CPU only.  Usage:
    python tools/bench_host.py [--grids 317,632] [--threads 0]
"""
import argparse
import json
import os
import pathlib
import subprocess
import sys
import tempfile

ROOT = pathlib.Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
import pathtracercuda_amd as pa  # noqa: E402


def load(path, threads):
    if threads:
        os.environ["PT_BVH_THREADS"] = str(threads)
    else:
        os.environ.pop("PT_BVH_THREADS", None)
    best = None
    for _ in range(3):
        s = pa.Scene(path, 1920, 1080)
        t = s.timing()
        if best is None or t["parse_ms"] + t["bvh_ms"] < best["parse_ms"] + best["bvh_ms"]:
            best = dict(t, objects=s.object_count, nodes=s.node_count, depth=s.bvh_depth)
            nodes = bytes(s.bvh()[0])
    return best, nodes


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--grids", default="317,632", help="stress-scene grid sizes (objects = grid^2)")
    ap.add_argument("--threads", type=int, default=0, help="BVH threads for the parallel run (0 = all cores)")
    a = ap.parse_args()
    scenes = [("cornell_box", ROOT / "scenes/cornell_box.scene.json"),
              ("generated_scene", ROOT / "scenes/generated_scene.scene.json")]
    tmp = tempfile.mkdtemp()
    for g in [int(x) for x in a.grids.split(",") if x]:
        p = pathlib.Path(tmp) / f"stress_{g}.json"
        subprocess.run([sys.executable, str(ROOT / "tools/make_stress_scene.py"), str(p), "--grid", str(g)],
                       check=True, capture_output=True)
        scenes.append((f"stress_{g * g}", p))
    out = {"cpus": os.cpu_count(), "scenes": {}}
    for name, path in scenes:
        seq, n_seq = load(path, 1)
        par, n_par = load(path, a.threads)
        assert n_seq == n_par, f"{name}: parallel BVH differs from sequential"
        out["scenes"][name] = {"objects": seq["objects"], "nodes": seq["nodes"], "depth": seq["depth"],
                               "json_bytes": os.path.getsize(path),
                               "parse_ms": round(min(seq["parse_ms"], par["parse_ms"]), 2),
                               "bvh_ms_sequential": round(seq["bvh_ms"], 2), "bvh_ms_parallel": round(par["bvh_ms"], 2)}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
