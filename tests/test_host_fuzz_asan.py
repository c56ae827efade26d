"""Randomised robustness of the host-only request helpers (omr_request.cpp, omr_host.cpp) under
AddressSanitizer + UBSan: tools/fuzz_host.cpp drives ImageRegionCtx / ShapeMaskCtx parsing,
createRenderingDef + updateSettings, getRegionDef / checkPlaneDef at the int32 edges,
splitHTMLColor and .lut parsing with hostile inputs.  CPU only; built here with g++."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "omero-ms-image-region_amd", "csrc")


@pytest.fixture(scope="module")
def fuzz_bin(tmp_path_factory):
    if shutil.which("g++") is None:
        pytest.skip("g++ not available")
    out = str(tmp_path_factory.mktemp("fuzz") / "fuzz_host")
    cmd = ["g++", "-std=c++17", "-O1", "-g", "-fsanitize=address,undefined", "-fno-sanitize-recover=all",
           "-static-libasan", "-I" + os.path.join(ROOT, "include"), os.path.join(ROOT, "tools", "fuzz_host.cpp"),
           os.path.join(CSRC, "omr_request.cpp"), os.path.join(CSRC, "omr_host.cpp"), "-o", out]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-4000:]
    return out


@pytest.mark.parametrize("seed", [1, 2])
def test_host_helpers_fuzz_sanitized(fuzz_bin, seed):
    iters = os.environ.get("OMR_HOST_FUZZ_ITERS", "5000")
    r = subprocess.run([fuzz_bin, iters, str(seed)], capture_output=True, text=True, timeout=600,
                       env=dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=0",
                                UBSAN_OPTIONS="print_stacktrace=1"))
    assert r.returncode == 0, (r.stdout[-2000:], r.stderr[-4000:])
    assert "iterations clean" in r.stdout
