"""The oracle against the analytic KATs of tests/kat.py (sky mapping and bilinear filter, GGX /
Lambert+GGX / Lambert white furnace).  The reference's published render pins only cornell's
Lambert/emissive light transport, so these pin the oracle's restatement of the rest to
independently integrated expectations.  The GPU runs the same cases (tests/test_gpu_kat.py)."""
import pytest

import kat
from oracle import pyoracle as po


def test_oracle_sky_only_kat(tmp_path):
    p, tex = kat.sky_case(tmp_path)
    W, H, spp = 24, 16, 512
    sc = po.load_scene(p, W, H)
    r = po.OracleRenderer(sc, W, H)
    r.render(sc.camera, 8, True, chunks=spp // 8)
    kat.check_sky(r.accum / spp, tex, W, H, spp, "oracle sky")


@pytest.mark.parametrize("mtype,rough,metal", kat.FURNACE_CASES)
def test_oracle_white_furnace(tmp_path, mtype, rough, metal):
    W, H, spp = 16, 16, 512
    p = kat.furnace_case(tmp_path, mtype, rough, metal)
    sc = po.load_scene(p, W, H)
    r = po.OracleRenderer(sc, W, H)
    r.render(sc.camera, 8, True, chunks=spp // 8)
    kat.check_furnace(r.accum / spp, kat.furnace_expectation(W, H, mtype, rough, metal), f"oracle {mtype} r={rough}")
