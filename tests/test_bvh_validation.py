"""Host validation of caller BVHs (pt_set_scene): the LDS stack-row bound over the reachable tree.

ADVICE r04: the bound was computed in node-array order over every node, so an unreachable interior
node naming a reachable child could overwrite that child's pending count and undercount the rows the
walks write.  bvh_edit.py builds such a BVH; the GPU half (test_gpu_parity.py::
test_orphan_node_bvh_renders_exactly) renders it against the oracle.
"""
from oracle import pyoracle as po
import bvh_edit as be


def scene_nodes(osc):
    return [(tuple(osc.nodes[i].bmin), tuple(osc.nodes[i].bmax), int(osc.nodes[i].offset),
             int(osc.nodes[i].primitiveCountAxis)) for i in range(osc.node_count)]


def orphan_caterpillar(osc, n=30, p=30):
    cat = be.caterpillar(be.leaves_of(scene_nodes(osc)), n)
    return cat, be.insert_orphan(cat, p)


def test_orphan_lowers_the_array_order_bound_only(scenes):
    osc = po.load_scene(scenes / "generated_scene.scene.json", 64, 64)
    nodes = scene_nodes(osc)
    assert be.stack_rows_array(nodes) == be.stack_rows_tree(nodes)   # the same on a proper tree
    cat, bad = orphan_caterpillar(osc)
    assert be.stack_rows_tree(cat) == be.stack_rows_array(cat) == 29    # n - 1 interior nodes in a chain
    assert be.stack_rows_tree(bad) == 29
    assert be.stack_rows_array(bad) <= 20, "the orphan must undercount the array-order bound"
