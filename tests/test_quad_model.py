"""CPU model of the 4-wide child-box walk (pt_kernels.hip walk_interior_quad, pt_set_scene's qnodes).

The kernel's 4-wide records and its walk are restated here in float32 numpy scalars and run against
the reference's hitBVH (trace.cu:28-98, AABB.inl:22-44 with its early exits) on the bench scene's
host-built BVH: for every ray the sequence of primitive tests must be the reference's, with t_max
lowered by a deterministic stand-in for the primitive test (so culling after hits is exercised).
Rays include axis-parallel directions (1/d infinite on two axes, the NaN-skipping slab form) and
origins on box faces.  The GPU parity suite checks the kernel itself bit for bit.
"""
import pathlib

import numpy as np
import pytest

import pathtracercuda_amd as pa

F = np.float32
INF = F(np.inf)
T_MIN = F(0.001)
PAIR = 1 << 23                  # pair word: PAIR | 2 r + h; landing word: r | split axis << 20


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


def build_quads(nodes):
    """pt_set_scene's qnodes: per even-depth interior node two halves of (L box, R box, wL, wR, axis
    bit); a landing word carries its node's split axis at bit 20; empty slot R of a leaf side =
    [+inf, +inf]^3."""
    n = len(nodes)
    odd = [0] * n
    qrec = [None] * n
    q = 0
    for i in range(n):
        if nodes[i].primitive_count_axis >> 16:
            continue
        for c in (i + 1, nodes[i].offset):
            odd[c] = odd[i] ^ 1
            cmin, cmax = box(nodes[c])
            pmin, pmax = box(nodes[i])
            assert (cmin >= pmin).all() and (cmax <= pmax).all()
        if not odd[i]:
            qrec[i] = q
            q += 1

    def word(i):
        cnt = nodes[i].primitive_count_axis >> 16
        return (cnt << 24) | nodes[i].offset if cnt else qrec[i] | (((nodes[i].primitive_count_axis >> 8) & 0xff) << 20)

    recs = [None] * q
    empty = (np.full(3, INF, F), np.full(3, INF, F))
    for i in range(n):
        if qrec[i] is None:
            continue
        halves = []
        for c in (i + 1, nodes[i].offset):
            if nodes[c].primitive_count_axis >> 16:
                halves.append((box(nodes[c]), empty, word(c), 0xffffffff, 0))
            else:
                halves.append((box(nodes[c + 1]), box(nodes[nodes[c].offset]), word(c + 1), word(nodes[c].offset),
                               1 << ((nodes[c].primitive_count_axis >> 8) & 0xff)))
        recs[qrec[i]] = halves
    return recs, word(0)


def cb_pair(half, o, d, negmask, tmax):
    """pt_kernels.hip cb_pair: hit flags at t_max, and the t_max-free 'box meets the ray' flags that
    decide what is kept for later."""
    (lb, rb, wl, wr, axis) = half
    lol, xl = lo_x(*lb, o, d)
    lor, xr = lo_x(*rb, o, d)
    isneg = (negmask & axis) != 0
    gl, gr = xl > lol, xr > lor
    hl = gl and tmax > lol
    hr = gr and tmax > lor
    takel = hl and (not hr or not isneg)
    return {"push": (hr and gl) if isneg else (hl and gr), "any": hl or hr,
            "wNext": wl if takel else wr, "loNext": lol if takel else lor,
            "wF": wl if isneg else wr, "loF": lol if isneg else lor,
            "gBoth": gl and gr, "gAny": gl or gr, "wG": wl if gl else wr, "loG": lol if gl else lor,
            "loMin": min(lol, lor)}


def quad_walk(recs, root_word, root_box, nodes, o, d, ray_id):
    negmask = (d[0] < 0) | ((d[1] < 0) << 1) | ((d[2] < 0) << 2)
    tests, stack, tmax = [], [], F(np.finfo(np.float32).max)
    lo0, x0 = lo_x(*root_box, o, d)
    if not (x0 > lo0 and tmax > lo0):
        return tests
    cur = root_word

    def pop():
        while stack:
            w, lo = stack.pop()
            if tmax > lo:
                return w
        return None

    while cur is not None:
        if cur >> 24 == 0:
            pair = (cur & PAIR) != 0
            r = (cur & ((1 << 21) - 1)) >> 1 if pair else cur & ((1 << 20) - 1)
            halves = recs[r]
            ha, hb = cb_pair(halves[0], o, d, negmask, tmax), cb_pair(halves[1], o, d, negmask, tmax)
            near_b = (cur & 1) != 0 if pair else ((negmask >> ((cur >> 20) & 3)) & 1) != 0
            nr, fr = (hb, ha) if near_b else (ha, hb)
            far_on = not pair and fr["any"]
            if nr["any"]:
                if not pair and fr["gAny"]:
                    if fr["gBoth"]:
                        stack.append((PAIR | (2 * r + (0 if near_b else 1)), fr["loMin"]))
                    else:
                        stack.append((fr["wG"], fr["loG"]))
                sd = nr
            elif far_on:
                sd = fr
            else:
                cur = pop()
                continue
            if sd["push"]:
                stack.append((sd["wF"], sd["loF"]))
            cur = sd["wNext"]
        else:
            off, cnt = cur & 0xffffff, cur >> 24
            for i in range(cnt):
                tests.append(off + i)
                t = prim_stub(off + i, ray_id, tmax)
                if t is not None:
                    tmax = t
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


def cb_walk(nodes, o, d, ray_id):
    """The 2-wide child-box walk (walk_interior / traverse_cb): both children tested at the parent's
    visit, the far child kept by cb_pair's `push` and re-tested (t_max > lo) when popped."""
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
            for i in range(cnt):
                tests.append(n.offset + i)
                t = prim_stub(n.offset + i, ray_id, tmax)
                if t is not None:
                    tmax = t
            cur = pop()
            continue
        a, b = cur + 1, n.offset
        ch = cb_pair((box(nodes[a]), box(nodes[b]), a, b, 1 << ((n.primitive_count_axis >> 8) & 0xff)), o, d, negmask,
                     tmax)
        if ch["push"]:
            stack.append((ch["wF"], ch["loF"]))
        cur = ch["wNext"] if ch["any"] else pop()
    return tests


@pytest.mark.parametrize("rise", [False, True])
@pytest.mark.parametrize("scene,nrays", [("generated_scene", 1500), ("cornell_box", 800), ("test_shapes", 400)])
def test_child_box_walks_match_reference_order(scene, nrays, rise):
    """Both shipped walks (2-wide and 4-wide) against hitBVH, also when t_max rises mid-traversal
    (the sphere's far-root quirk): pending children are dropped only for t_max-free reasons."""
    RISE[0] = rise
    try:
        root = pathlib.Path(__file__).resolve().parents[1]
        sc = pa.Scene(str(root / "scenes" / f"{scene}.scene.json"), 64, 64)
        nodes = list(sc.bvh()[0])
        recs, root_word = build_quads(nodes)
        for k, (o, d) in enumerate(rays(nodes, nrays, 11)):
            want = reference_walk(nodes, o, d, k)
            assert cb_walk(nodes, o, d, k) == want, ("2-wide", k)
            assert quad_walk(recs, root_word, box(nodes[0]), nodes, o, d, k) == want, ("4-wide", k)
    finally:
        RISE[0] = False


@pytest.mark.parametrize("scene,nrays", [("generated_scene", 1500), ("cornell_box", 800), ("test_shapes", 400)])
def test_quad_walk_matches_reference_order(scene, nrays):
    root = pathlib.Path(__file__).resolve().parents[1]
    sc = pa.Scene(str(root / "scenes" / f"{scene}.scene.json"), 64, 64)
    nodes, _ = sc.bvh()
    nodes = list(nodes)
    recs, root_word = build_quads(nodes)
    n_leaf_sides = sum(1 for r in recs for h in r if h[3] == 0xffffffff)
    assert len(recs) >= 1
    nonempty = 0
    for k, (o, d) in enumerate(rays(nodes, nrays, 7)):
        want = reference_walk(nodes, o, d, k)
        got = quad_walk(recs, root_word, box(nodes[0]), nodes, o, d, k)
        assert got == want, (k, o, d, want[:10], got[:10])
        nonempty += bool(want)
    assert nonempty > nrays // 10, nonempty
    assert n_leaf_sides >= 0
