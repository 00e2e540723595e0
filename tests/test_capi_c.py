"""The C ABI from C: include/cfd2_amd.h compiles as strict C99 (-pedantic
-Werror) and a C program links against the in-tree library (CPU); on a GPU it
generates a mesh, steps the solver, reads the fields and saves a checkpoint
(tests/native/abi_smoke.c)."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIBDIR = os.path.join(ROOT, "cfd-demo2_amd", "cfd2_amd", "_lib")


def _build(tmp_path):
    exe = str(tmp_path / "abi_smoke")
    cmd = ["gcc", "-std=c99", "-Wall", "-Wextra", "-Werror", "-pedantic",
           os.path.join(ROOT, "tests", "native", "abi_smoke.c"), "-o", exe, f"-L{LIBDIR}", "-lcfd2_amd",
           f"-Wl,-rpath,{LIBDIR}", "-lm"]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr[-3000:]
    return exe


@pytest.mark.skipif(shutil.which("gcc") is None, reason="gcc not available")
def test_header_is_c99_and_links(tmp_path):
    assert os.path.exists(os.path.join(LIBDIR, "libcfd2_amd.so")), "build the library first"
    _build(tmp_path)


@pytest.mark.gpu
def test_c_program_steps_the_solver(tmp_path):
    exe = _build(tmp_path)
    r = subprocess.run([exe, str(tmp_path / "s.state")], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr[-3000:]
    assert ": ok" in r.stdout
    assert (tmp_path / "s.state").stat().st_size > 512
