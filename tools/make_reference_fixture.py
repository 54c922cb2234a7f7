"""Derive a statistical fixture from the reference's own published render.

cornell_box_4096spp.png (reference PathtracerCUDA/, 1024x1024, windowed mode = 1 spp per render()
call, so correctly normalised; tonemap.cu:16-26: Reinhard c/(c+1), gamma 1/2.2, truncation to 8
bits; saved with a vertical flip, main.cpp:184) is inverted back to linear radiance per pixel and
averaged over a 32x32 grid of 32x32-pixel blocks.  Blocks are indexed in accumulation-buffer order
(row 0 = bottom of the picture).  The file is data derived from the reference's output (no
reference source is copied); tests compare the oracle's and the GPU's normalised accumulation
against it with a loose tolerance (the reference had earth.png, which is absent here, so blocks
touching the textured sphere are masked).
"""
import json
import pathlib
import sys

import numpy as np
from PIL import Image

SRC = pathlib.Path("/root/reference/PathtracerCUDA/cornell_box_4096spp.png")
DST = pathlib.Path(__file__).resolve().parents[1] / "tests" / "golden" / "cornell_ref_blocks.json"
GRID = 32


def main() -> int:
    img = np.asarray(Image.open(SRC).convert("RGB"), dtype=np.float64)
    h, w, _ = img.shape
    img = img[::-1]                                   # undo stbi_flip_vertically_on_write
    g = ((img + 0.5) / 255.0) ** 2.2                  # undo gamma (mid-bin of the truncated value)
    g = np.clip(g, 0.0, 0.995)
    lin = g / (1.0 - g)                               # undo Reinhard
    bh, bw = h // GRID, w // GRID
    blocks = lin.reshape(GRID, bh, GRID, bw, 3).mean(axis=(1, 3))
    DST.parent.mkdir(parents=True, exist_ok=True)
    DST.write_text(json.dumps({
        "source": "reference PathtracerCUDA/cornell_box_4096spp.png",
        "width": w, "height": h, "grid": GRID,
        "note": "linear radiance block means, row 0 = bottom (accumulation order)",
        "blocks": np.round(blocks, 6).tolist(),
    }) + "\n")
    print(f"wrote {DST}")
    return 0


if __name__ == "__main__":
    sys.exit(main())
