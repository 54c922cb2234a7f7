"""Store the reference's published cornell render as a pixel fixture (tests/golden/*_ref8.npz).

The reference ships two renders made by its own windowed loop (main.cpp:387-399: one render(cam, 1)
call per frame, so the tonemap divisor is the sample count; tonemap.cu:16-26; saved with a vertical
flip, main.cpp:184).  This keeps their 8-bit RGB values, un-flipped into accumulation-buffer order
(row 0 = bottom), so tests compare them with our own tonemap of the same render pixel for pixel.
These are output data of the reference, not source.  Only the cornell render is kept: the
generated_scene render used the reference's skybox.hdr and earth.png, which its checkout lacks
(our sky is synthetic), so no test can compare it.  Run here (the reference is not on the GPU box):
    python tools/make_png_fixture.py
"""
import pathlib

import numpy as np
from PIL import Image

REF = pathlib.Path("/root/reference/PathtracerCUDA")
DST = pathlib.Path(__file__).resolve().parents[1] / "tests" / "golden"


def main() -> None:
    for name in ("cornell_box_4096spp",):
        img = np.asarray(Image.open(REF / f"{name}.png").convert("RGB"), dtype=np.uint8)[::-1]
        out = DST / f"{name}_ref8.npz"
        np.savez_compressed(out, rgb=np.ascontiguousarray(img), source=f"reference PathtracerCUDA/{name}.png")
        print(f"wrote {out} {img.shape} {out.stat().st_size} B")


if __name__ == "__main__":
    main()
