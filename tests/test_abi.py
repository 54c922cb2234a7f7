"""The C ABI libraries load without a GPU and export every entry point include/*.h declares."""
import re

import pytest

import pathtracercuda_amd as pa
from pathtracercuda_amd import _native as N


def declared(header_text):
    body = "\n".join(l for l in header_text.splitlines() if not l.lstrip().startswith("#"))
    return set(re.findall(r"PT_API\s+[^;(]*?\b(\w+)\s*\(", body))


@pytest.mark.parametrize("header,lib,table", [("pt_hip.h", "hip", "_HIP_SYMBOLS"), ("pt_host.h", "host", "_HOST_SYMBOLS")])
def test_every_declared_symbol_is_exported_and_bound(root, header, lib, table):
    names = declared((root / "include" / header).read_text())
    assert len(names) >= 10
    L = getattr(N, lib)()
    for n in names:
        assert hasattr(L, n), f"{n} declared in {header} but not exported"
    assert names == set(getattr(N, table)), "Python binding table out of sync with the header"


def test_no_gpu_calls_fail_cleanly():
    # pt_create without a device must return an error code, never crash (CPU container)
    if pa.device_count() > 0:
        pytest.skip("GPU present")
    with pytest.raises(pa.PathtracerError):
        pa.Pathtracer(8, 8)


def test_hip_library_is_gfx950(tmp_path):
    # llvm-objdump --offloading extracts the device bundles next to its input: run it on a copy in
    # a temporary directory so nothing lands in the package's lib/
    import shutil
    import subprocess
    lib = tmp_path / N.HIP_LIB.name
    shutil.copy(N.HIP_LIB, lib)
    out = subprocess.run(["/opt/rocm/lib/llvm/bin/llvm-objdump", "--offloading", str(lib)],
                         capture_output=True, text=True, cwd=tmp_path)
    text = out.stdout + out.stderr
    assert "gfx950" in text
    assert not list(N.HIP_LIB.parent.glob(N.HIP_LIB.name + ".*")), "bundle files in the package lib/"


@pytest.mark.parametrize("order", ["native_first", "torch_first"])
def test_import_order_keeps_one_runtime(root, order):
    # ADVICE/VERDICT r05: libpt_hip.so loaded before torch used to map torch's and /opt/rocm's HIP
    # runtimes side by side and abort at exit ("double free or corruption", rc 134).  _native.hip()
    # imports torch first, so either order ends with one runtime and a clean exit.
    import subprocess
    import sys
    steps = ["from pathtracercuda_amd import _native as N", "N.hip()", "import torch"]
    if order == "torch_first":
        steps = [steps[2]] + steps[:2]
    code = "\n".join(steps + ["N.check_single_runtime()", "print(len(N.mapped_hip_runtimes()))"])
    out = subprocess.run([sys.executable, "-c", code], cwd=root, capture_output=True, text=True, timeout=300)
    assert out.returncode == 0, out.stderr[-2000:]
    assert out.stdout.split()[-1] == "1"
