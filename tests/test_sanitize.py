"""Host sanitizers: the oracle, the product's host mesh code
(cut-cell, Voronoi, Delaunay generators) built with AddressSanitizer + UBSan
(+ leak detection) straight from the sources and run on small meshes, one and
three ranks (oracle/sanitize_main.cpp).  CPU only."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.skipif(shutil.which("g++") is None, reason="g++ not available")
def test_oracle_and_mesh_code_under_asan_ubsan(tmp_path):
    exe = str(tmp_path / "sanitize")
    srcs = [os.path.join(ROOT, p) for p in ("oracle/sanitize_main.cpp", "oracle/oracle.cpp",
                                            "cfd-demo2_amd/csrc/mesh/cut_cell.cpp",
                                            "cfd-demo2_amd/csrc/mesh/voronoi.cpp")]
    cmd = ["g++", "-O1", "-g", "-std=c++17", "-fopenmp", "-ffp-contract=off", "-fsanitize=address,undefined",
           "-fno-omit-frame-pointer", "-fno-sanitize-recover=undefined", *srcs, "-o", exe]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=0", UBSAN_OPTIONS="print_stacktrace=1")
    r = subprocess.run([exe], capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    assert r.stdout.count(": ok") == 8, r.stdout


@pytest.mark.skipif(shutil.which("g++") is None or not os.path.isdir("/opt/rocm/include"),
                    reason="g++ / ROCm headers not available")
def test_host_setup_code_under_asan_ubsan(tmp_path):
    """The product's GPU-free host setup code: slab topology and halo plans for
    1-4 ranks, the host AMG hierarchy (tests/native/sanitize_host.cpp)."""
    exe = str(tmp_path / "sanitize_host")
    srcs = [os.path.join(ROOT, p) for p in ("tests/native/sanitize_host.cpp", "cfd-demo2_amd/csrc/host/topology.cpp",
                                            "cfd-demo2_amd/csrc/host/amg_setup.cpp", "cfd-demo2_amd/csrc/host/dist.cpp",
                                            "cfd-demo2_amd/csrc/mesh/cut_cell.cpp",
                                            "cfd-demo2_amd/csrc/mesh/voronoi.cpp")]
    cmd = ["g++", "-O1", "-g", "-std=c++17", "-fopenmp", "-ffp-contract=off", "-fsanitize=address,undefined",
           "-fno-omit-frame-pointer", "-fno-sanitize-recover=undefined", "-D__HIP_PLATFORM_AMD__",
           "-I/opt/rocm/include", *srcs, "-o", exe]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1", UBSAN_OPTIONS="print_stacktrace=1")
    r = subprocess.run([exe], capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    # every mesh: 1 rank up to min(4, its reduction segments of 256 cells) ranks
    for mesh in ("cut-cell step", "voronoi channel", "delaunay channel"):
        assert all(f"{mesh}: " in r.stdout and f", {R} rank(s):" in r.stdout for R in (1, 2, 3)), r.stdout
    assert r.stdout.count(": ok") >= 9, r.stdout
