"""CPU model of the child-box walk (pt_kernels.hip cb_pair / walk_interior / repair_pending).

The kernel's walk -- both children tested at the parent's visit, the far child kept only when hit
at the current t_max, and the reference's pending set rebuilt when a leaf RAISES t_max (the
sphere's far-root quirk, Hittable.inl:158) -- is restated here in float32 numpy scalars and run
against the reference's hitBVH (trace.cu:28-98, AABB.inl:22-44 with its early exits) on the scenes'
host-built BVHs: for every ray the sequence of primitive tests must be the reference's.  The
primitive test is a deterministic stand-in that lowers t_max, and with RISE sometimes raises it.
Rays include axis-parallel directions (1/d infinite on two axes, the NaN-skipping slab form),
origins on box faces and rays aimed at leaves.  The GPU parity suite checks the kernel itself bit
for bit (and compares the child-box walk with the reference's control flow, variant 1, over whole frames).
"""
import pathlib

import numpy as np
import pytest

import pathtracercuda_amd as pa

F = np.float32
INF = F(np.inf)
T_MIN = F(0.001)


def box(n):
    return np.array(n.aabb_min, F), np.array(n.aabb_max, F)


def ref_hit(bmin, bmax, o, d, tmin, tmax):
    """AABB::hit (AABB.inl:22-44) with its early exits."""
    with np.errstate(all="ignore"):
        for a in range(3):
            inv = F(1.0) / d[a]
            t0 = (bmin[a] - o[a]) * inv
            t1 = (bmax[a] - o[a]) * inv
            if inv < 0:
                t0, t1 = t1, t0
            tmin = t0 if t0 > tmin else tmin
            tmax = t1 if t1 < tmax else tmax
            if tmax <= tmin:
                return False
    return True


def lo_x(bmin, bmax, o, d):
    """slab_lo_x (exact form): lo and X, both independent of t_max."""
    lo, hi = T_MIN, INF
    with np.errstate(all="ignore"):
        for a in range(3):
            inv = F(1.0) / d[a]
            t0 = (bmin[a] - o[a]) * inv
            t1 = (bmax[a] - o[a]) * inv
            if inv < 0:
                t0, t1 = t1, t0
            lo = t0 if t0 > lo else lo
            hi = t1 if t1 < hi else hi
    return lo, hi


RISE = [False]


def prim_stub(p, ray_id, tmax):
    """Deterministic stand-in for Hittable::hit: hits 30 % of the time, at a t below t_max -- or, with
    RISE set, sometimes ABOVE t_max, as the sphere's far-root quirk does (Hittable.inl:158: t1 is
    accepted when t0 <= t_min, whatever t_max is)."""
    h = (p * 2654435761 + ray_id * 40503) & 0xffffffff
    if h % 10 >= 3:
        return None
    if RISE[0] and h % 5 == 0 and tmax < 1e30:
        return F(float(tmax) * 1.5 + 0.5)
    t = F(T_MIN + (h >> 8) % 1000 / 1000.0 * min(float(tmax), 50.0))
    return t if T_MIN < t <= tmax else None


def reference_walk(nodes, o, d, ray_id):
    tests, stack, cur, tmax = [], [], 0, F(np.finfo(np.float32).max)
    while True:
        n = nodes[cur]
        bmin, bmax = box(n)
        if ref_hit(bmin, bmax, o, d, T_MIN, tmax):
            cnt = n.primitive_count_axis >> 16
            if cnt:
                for i in range(cnt):
                    tests.append(n.offset + i)
                    t = prim_stub(n.offset + i, ray_id, tmax)
                    if t is not None:
                        tmax = t
                if not stack:
                    break
                cur = stack.pop()
            else:
                neg = d[(n.primitive_count_axis >> 8) & 0xff] < 0
                stack.append(cur + 1 if neg else n.offset)
                cur = n.offset if neg else cur + 1
        else:
            if not stack:
                break
            cur = stack.pop()
    return tests


def first_prims(nodes):
    """First primitive under each node (pt_set_scene: child-box record Q3.w of the second child)."""
    first = [0] * len(nodes)
    for i in range(len(nodes) - 1, -1, -1):
        n = nodes[i]
        first[i] = n.offset if n.primitive_count_axis >> 16 else min(first[i + 1], first[n.offset])
    return first


def repair(nodes, first, o, d, negmask, leaf_off):
    """repair_pending: the reference's pending far children on the path to the leaf at leaf_off,
    left out when the ray does not meet their box at all."""
    stack, n = [], 0
    while not nodes[n].primitive_count_axis >> 16:
        a, b = n + 1, nodes[n].offset
        in_r = leaf_off >= first[b]
        neg = (negmask >> ((nodes[n].primitive_count_axis >> 8) & 0xff)) & 1
        other = a if in_r else b
        if in_r == bool(neg):                # the path took the near child
            lo, x = lo_x(*box(nodes[other]), o, d)
            if x > lo:
                stack.append((other, lo))
        n = b if in_r else a
    return stack


def cb_walk(nodes, first, o, d, ray_id, rise_all=False, rebuild=True):
    """The child-box walk: far child kept when hit now (or, rise_all, whenever the ray meets its
    box), re-tested (t_max > lo) when popped; the pending set rebuilt after a leaf raised t_max
    (rebuild=False: rounds 1-3, without it)."""
    negmask = (d[0] < 0) | ((d[1] < 0) << 1) | ((d[2] < 0) << 2)
    tests, stack, tmax = [], [], F(np.finfo(np.float32).max)
    lo0, x0 = lo_x(*box(nodes[0]), o, d)
    if not (x0 > lo0 and tmax > lo0):
        return tests
    cur = 0

    def pop():
        while stack:
            w, lo = stack.pop()
            if tmax > lo:
                return w
        return None

    while cur is not None:
        n = nodes[cur]
        cnt = n.primitive_count_axis >> 16
        if cnt:
            t_leaf = tmax
            for i in range(cnt):
                tests.append(n.offset + i)
                t = prim_stub(n.offset + i, ray_id, tmax)
                if t is not None:
                    tmax = t
            if tmax > t_leaf and rebuild and not rise_all:
                stack[:] = repair(nodes, first, o, d, negmask, n.offset)
            cur = pop()
            continue
        a, b = cur + 1, n.offset
        loa, xa = lo_x(*box(nodes[a]), o, d)
        lob, xb = lo_x(*box(nodes[b]), o, d)
        ha, hb = xa > loa and tmax > loa, xb > lob and tmax > lob
        neg = (negmask >> ((n.primitive_count_axis >> 8) & 0xff)) & 1
        near, far = (b, a) if neg else (a, b)
        hn, hf = (hb, ha) if neg else (ha, hb)
        lof, xf = (loa, xa) if neg else (lob, xb)
        if hn:
            if (xf > lof) if rise_all else hf:
                stack.append((far, lof))
            cur = near
        elif hf:
            cur = far
        else:
            cur = pop()
    return tests


def rays(nodes, n, seed):
    rng = np.random.default_rng(seed)
    bmin, bmax = box(nodes[0])
    leaves = [m for m in nodes if m.primitive_count_axis >> 16]
    out = []
    for k in range(n):
        o = (bmin + (bmax - bmin) * rng.uniform(-0.2, 1.2, 3)).astype(F)
        d = rng.normal(size=3).astype(F)
        if k % 5 == 1:                       # axis-parallel: two zero components, 1/d = +-inf
            d[np.arange(3) != k % 3] = 0.0
        if k % 7 == 2:                       # origin on a box face of a random node
            m = nodes[rng.integers(len(nodes))]
            o[k % 3] = np.array(m.aabb_min, F)[k % 3]
        if k % 2 == 0:                       # aimed at a random leaf's box: rays that reach primitives
            leaf = leaves[rng.integers(len(leaves))]
            lmin, lmax = box(leaf)
            d = (lmin + (lmax - lmin) * rng.uniform(0, 1, 3) - o).astype(F)
        d = (d / np.linalg.norm(d)).astype(F) if np.linalg.norm(d) > 0 else np.array([0, 1, 0], F)
        out.append((o, d))
    return out


@pytest.mark.parametrize("rise", [False, True])
@pytest.mark.parametrize("scene,nrays", [("generated_scene", 1500), ("cornell_box", 800), ("test_shapes", 400)])
def test_child_box_walk_matches_reference_order(scene, nrays, rise):
    """The kernel's rule (hit-now + rebuild after a rise) and the reference's (keep every far child
    the ray meets) give hitBVH's primitive-test sequence, also when t_max rises mid-traversal."""
    RISE[0] = rise
    try:
        root = pathlib.Path(__file__).resolve().parents[1]
        sc = pa.Scene(str(root / "scenes" / f"{scene}.scene.json"), 64, 64)
        nodes = list(sc.bvh()[0])
        first = first_prims(nodes)
        nonempty = 0
        for k, (o, d) in enumerate(rays(nodes, nrays, 11)):
            want = reference_walk(nodes, o, d, k)
            assert cb_walk(nodes, first, o, d, k) == want, ("hit-now + rebuild", k)
            assert cb_walk(nodes, first, o, d, k, rise_all=True) == want, ("keep every far child", k)
            nonempty += bool(want)
        assert nonempty > nrays // 4, nonempty
    finally:
        RISE[0] = False


def test_hit_now_rule_alone_misses_rises():
    """Without the rebuild, the hit-now rule leaves the reference's path when t_max rises (what rounds
    1-3 shipped): the model must see it, or the test above proves nothing."""
    RISE[0] = True
    try:
        root = pathlib.Path(__file__).resolve().parents[1]
        sc = pa.Scene(str(root / "scenes" / "generated_scene.scene.json"), 64, 64)
        nodes = list(sc.bvh()[0])
        first = first_prims(nodes)
        bad = 0
        for k, (o, d) in enumerate(rays(nodes, 1500, 11)):
            if cb_walk(nodes, first, o, d, k, rebuild=False) != reference_walk(nodes, o, d, k):
                bad += 1
        assert bad > 0
    finally:
        RISE[0] = False
