"""Import the reference's example scenes as canonical, minified JSON fixtures.

The reference scene files (PathtracerCUDA/cornell_box.json, generated_scene.json) are the inputs of
BASELINE.json configs C1-C4.  They are re-serialised (sorted keys, no whitespace) so the repo holds
the same data -- every float keeps its exact double value, every JSON integer stays an integer
(SceneLoader.cpp:163-171 only accepts JSON floats for roughness/metalness/fovy) -- without keeping a
byte copy of the reference files.  Run once from a container that has /root/reference.
"""
import json
import pathlib
import sys

SRC = pathlib.Path("/root/reference/PathtracerCUDA")
DST = pathlib.Path(__file__).resolve().parents[1] / "scenes"


def main() -> int:
    DST.mkdir(exist_ok=True)
    for name in ("cornell_box", "generated_scene"):
        data = json.loads((SRC / f"{name}.json").read_text())
        out = DST / f"{name}.scene.json"
        out.write_text(json.dumps(data, sort_keys=True, separators=(",", ":")) + "\n")
        print(f"wrote {out} ({len(data.get('objects', []))} objects)")
    return 0


if __name__ == "__main__":
    sys.exit(main())
