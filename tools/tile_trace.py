"""Schedule trace of one rank's share (pt_set_tile_trace; instrumented build, whose schedule rules are the
plain kernel's): for warm launches under each setting, every
tile's order position, start and duration (shader clock at 2.4 GHz; s_memtime is per CU and wraps at
2^32 cycles, so each CU's starts are zeroed at its first) and the CU / SIMD of the wave that ran it.  Saves an .npz for offline analysis and prints the
tiles that end last.
    python tools/tile_trace.py [--n 8 --rank 2 --width 3840 --height 2160 --spp 4096]
                               [--settings 0,5120/5120/12240] [--out gpurun_out/trace.npz]
A setting is P3[/P2/P1]: priority bounds as in tools/prio_probe.py (0 = automatic).
"""
import argparse
import json
import pathlib
import sys

import numpy as np

ROOT = pathlib.Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
import pathtracercuda_amd as pa  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--n", type=int, default=8)
ap.add_argument("--rank", type=int, default=2)
ap.add_argument("--width", type=int, default=3840)
ap.add_argument("--height", type=int, default=2160)
ap.add_argument("--spp", type=int, default=4096)
ap.add_argument("--settings", default="0")
ap.add_argument("--out", default=str(ROOT / "gpurun_out/trace.npz"))
ap.add_argument("--scene", default=str(ROOT / "scenes/generated_scene.scene.json"))
a = ap.parse_args()
settings = a.settings.split(",")
pt = pa.Pathtracer(a.width, a.height, row_offset=a.rank, row_stride=a.n, band_rows=8)
cam = pt.load_scene(a.scene)
chunks = a.spp // 8
for _ in range(2):
    pt.render_raw(cam, 8, chunks, True)                  # cold start, then its order rebuild
ref = pt.tile_costs().ravel().astype(np.float64)
order = np.argsort(-ref, kind="stable")                  # the order the warm launches run in
n = ref.size
pos_of = np.empty(n, np.int64)
pos_of[order] = np.arange(n)
pt.set_tile_trace(True)
save = {"pos_of": pos_of}
for k in settings:
    b = [int(x) for x in k.split("/")]
    if b == [0]:
        pt.set_issue_priority(0)
    else:
        b = (b + [max(b[-1], n // 2), max(b[-1], n - n // 4)])[:3]
        pt.set_issue_priority(2, *b)
    ms = pt.render_instrumented(cam, 8, chunks, True)["ms"]
    tr = pt.tile_trace().reshape(-1, 2)
    dur = pt.tile_costs().ravel().astype(np.float64) / 2.4e6
    hw = tr[:, 1]
    xcc, hwid = hw >> 16, hw & 0xffff
    simd = (hwid >> 4) & 3
    cu = (xcc << 8) | (((hwid >> 13) & 7) << 5) | (((hwid >> 12) & 1) << 4) | ((hwid >> 8) & 15)
    W = 2.0 ** 32 / 2.4e6
    st = tr[:, 0].astype(np.float64) / 2.4e6
    for x in np.unique(cu):                              # zero each CU's clock at its first tile start
        m = np.where(cu == x)[0]
        v = np.sort(st[m] % W)
        i = int(np.argmax(np.diff(np.r_[v, v[0] + W])))
        st[m] = (st[m] - v[(i + 1) % len(v)]) % W
    end = st + dur
    k = k.replace("/", "_")
    save.update({f"start_{k}": st, f"dur_{k}": dur, f"cu_{k}": cu, f"simd_{k}": simd})
    last = np.argsort(-end)[:12]
    print(json.dumps({"setting": k, "ms": round(ms, 2), "max_end_ms": round(float(end.max()), 1),
                      "last": [[int(pos_of[i]), round(float(st[i]), 1), round(float(dur[i]), 1), int(cu[i]), int(simd[i])]
                               for i in last]}), flush=True)
np.savez_compressed(a.out, **save)
