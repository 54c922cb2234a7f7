"""BVH surgery for the validation tests (pure Python, no native code).

A node is (bmin, bmax, offset, primitiveCountAxis) in the reference's layout (BVH.h:6-11): an
interior node's first child is the next node and its second child is `offset`; a leaf holds
primitiveCountAxis >> 16 primitives from `offset`.

caterpillar() chains a scene's leaves into a deep tree (every interior node: a leaf first, the rest
second), so the walk's pending far children grow with depth along one octant.  insert_orphan() then
adds an unreachable interior node that names a deep reachable node as its first child: an algorithm
that walks the node ARRAY instead of the tree from the root lets the orphan overwrite that child's
values -- the stack-row bound of pt_set_scene did that before round 5.  The tree
reachable from the root, and so every render, is unchanged.

stack_rows_array() / stack_rows_tree() restate the two forms of that bound (the LDS stack rows the
child-box walks need: max over the 8 direction octants of pend(v) + 1 over interior v, where pend(v) =
the far children pending when v is visited, trace.cu:66-77).
"""
from __future__ import annotations

from typing import List, Sequence, Tuple

Node = Tuple[Tuple[float, float, float], Tuple[float, float, float], int, int]


def _interior(n: Node) -> bool:
    return (n[3] >> 16) == 0


def stack_rows_array(nodes: Sequence[Node]) -> int:
    """The pre-round-5 form: pend propagated in array order over ALL nodes."""
    pend = [0] * len(nodes)
    need = 1
    for o in range(8):
        pend[0] = 0
        for i, (_, _, off, pca) in enumerate(nodes):
            if (pca >> 16) != 0:
                continue
            neg = (o >> ((pca >> 8) & 0xFF)) & 1
            a, b = i + 1, off
            pend[b if neg else a] = pend[i] + 1
            pend[a if neg else b] = pend[i]
            need = max(need, pend[i] + 1)
    return need


def stack_rows_tree(nodes: Sequence[Node]) -> int:
    """The round-5 form: pend carried down the root DFS (reachable nodes only)."""
    need = 1
    for o in range(8):
        st = [(0, 0)]
        while st:
            i, p = st.pop()
            _, _, off, pca = nodes[i]
            if (pca >> 16) != 0:
                continue
            need = max(need, p + 1)
            neg = (o >> ((pca >> 8) & 0xFF)) & 1
            a, b = i + 1, off
            st.append((b if neg else a, p + 1))
            st.append((a if neg else b, p))
    return need


def _union(boxes):
    lo = tuple(min(b[0][k] for b in boxes) for k in range(3))
    hi = tuple(max(b[1][k] for b in boxes) for k in range(3))
    return lo, hi


def leaves_of(nodes: Sequence[Node]) -> List[Node]:
    """The leaves in DFS order (first child before second)."""
    out, st = [], [0]
    while st:
        i = st.pop()
        n = nodes[i]
        if _interior(n):
            st.append(n[2])
            st.append(i + 1)
        else:
            out.append(n)
    return out


def caterpillar(leaves: Sequence[Node], n: int, axis: int = 2) -> List[Node]:
    """n leaves (consecutive runs of `leaves`, which must cover consecutive primitive ranges in
    order) chained as I0 -> (L0, I1), I1 -> (L1, I2), ..., split axis `axis`: depth n."""
    groups = [list(leaves[k * len(leaves) // n:(k + 1) * len(leaves) // n]) for k in range(n)]
    cl = []
    for g in groups:
        lo, hi = _union([(x[0], x[1]) for x in g])
        off = g[0][2]
        cnt = sum(x[3] >> 16 for x in g)
        assert all(g[j + 1][2] == g[j][2] + (g[j][3] >> 16) for j in range(len(g) - 1)), "leaves not consecutive"
        assert cnt < 256
        cl.append((lo, hi, off, cnt << 16))
    out: List[Node] = []
    for k in range(n - 1):
        lo, hi = _union([(x[0], x[1]) for x in cl[k:]])
        out.append((lo, hi, 2 * k + 2, axis << 8))
        out.append(cl[k])
    out.append(cl[n - 1])
    return out


def insert_orphan(nodes: Sequence[Node], p: int) -> List[Node]:
    """Insert an unreachable interior node at index p (node p - 1 must be a leaf, so nothing names p
    as a first child); its children are the shifted old node p and that node's second child."""
    assert p >= 1 and not _interior(nodes[p - 1]) and _interior(nodes[p])
    out: List[Node] = []
    for i, (lo, hi, off, pca) in enumerate(nodes):
        if i == p:
            out.append((lo, hi, nodes[p][2] + 1, pca & 0xFF00))   # orphan: first child p + 1 (= old p)
        out.append((lo, hi, (off + 1 if off >= p else off) if (pca >> 16) == 0 else off, pca))
    return out


def append_malformed_orphans(nodes: Sequence[Node]) -> List[Node]:
    """Append unreachable nodes whose fields would index out of bounds if read: an
    interior node with a second child far past the array, a leaf of 300 primitives past the primitive
    array, and an interior node at the last index (its first child i + 1 does not exist).  Nothing
    reachable from the root changes."""
    lo, hi = nodes[0][0], nodes[0][1]
    n = len(nodes)
    return list(nodes) + [(lo, hi, n + 1000, 0), (lo, hi, 1 << 23, 300 << 16), (lo, hi, 1, 1 << 8)]


def rise_pair_bvh(aabbs) -> Tuple[List[Node], List[int]]:
    """Caller BVH over scenes/rise_pair.scene.json's objects (file order: 0 dome, 1 sphere A, 2 wall B
    behind A; camera looking down -z), returns (nodes, object index of each primitive slot):

        0 R  split z -> first 1 (N), second 4 (leaf A)      d.z < 0: near = second = A
        1 N  split z -> first 2 (leaf B), second 3 (leaf dome)   near = second = dome
        2 leaf B   3 leaf dome   4 leaf A                    primitives [B, dome, A]: DFS order

    A ray that hits A: R pushes N, A's leaf sets t_max = tA; N is popped, its far child B fails at tA
    (B lies behind A) and is not kept by the hit-now rule, the dome's leaf returns its far root t1 >
    tA (Hittable.inl:152-158, the ray starts inside) and RAISES t_max; the reference then pops B's
    leaf, which passes at t1, and B's hit at tB < t1 wins (trace.cu:48-98).  Without the rebuild of
    the pending set the dome would win."""
    box = [(tuple(a[:3]), tuple(a[3:])) for a in aabbs]
    order = [2, 0, 1]                                         # slots: B, dome, A
    leaf = {o: (box[o][0], box[o][1], slot, 1 << 16) for slot, o in enumerate(order)}
    n_lo, n_hi = _union([box[2], box[0]])
    r_lo, r_hi = _union([box[0], box[1], box[2]])
    nodes = [(r_lo, r_hi, 4, 2 << 8), (n_lo, n_hi, 3, 2 << 8), leaf[2], leaf[0], leaf[1]]
    return nodes, order
