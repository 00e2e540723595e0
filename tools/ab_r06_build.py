"""Builds the libraries of the round-6 C2 regression A/B (VERDICT r05 "Next"
item 3; run on the CPU host before tools/gpu_ab_r06_regression.sh):
  r04     the round-4 tree (git df89dc708330, the BENCH_r04 head) exported to
          abtrees/r04 and built there with its own build (its own bench.py and
          package, since the ABI grew since then)
  nokpre  the current sources without -amdgpu-kernarg-preload-count=16
  nohead  the current sources with commit 0b05cfe (the smoother's leading
          preloaded arguments) reverted in kernels.hip
The current in-tree library is "base".  Variant libraries land in
cfd-demo2_amd/cfd2_amd/_lib/ab/ (they travel with gpurun; delete after)."""
import os
import shutil
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import __graft_entry__ as g  # noqa: E402

AB = os.path.join(g.LIB_DIR, "ab")
os.makedirs(AB, exist_ok=True)


def sh(cmd, **kw):
    print("+", cmd if isinstance(cmd, str) else " ".join(cmd), flush=True)
    subprocess.run(cmd, check=True, **kw)


def r04():
    dst = os.path.join(ROOT, "abtrees", "r04")
    if os.path.exists(dst):
        shutil.rmtree(dst)
    os.makedirs(dst)
    sh(f"git -C {ROOT} archive df89dc708330 cfd-demo2_amd include __graft_entry__.py bench.py tests | tar -x -C {dst}",
       shell=True)
    sh([sys.executable, "-c", "import __graft_entry__ as g; g.build_product(force=True)"], cwd=dst)


def nokpre():
    flags = [f for f in g.HIP_FLAGS if "kernarg-preload" not in f]
    i = flags.index("-mllvm") if "-mllvm" in flags else -1
    if i >= 0 and (i + 1 == len(flags) or flags[i + 1].startswith("-")):
        flags.pop(i)
    g.HIP_FLAGS[:] = flags
    lib = os.path.join(g.LIB_DIR, "variants", "libcfd2_amd_nokpre.so")
    g.build_product(lib=lib, obj_dir=os.path.join(g.OBJ_DIR, "v_nokpre"), force=True)
    shutil.copy(lib, os.path.join(AB, "libcfd2_amd_nokpre.so"))


def nohead():
    tmp = "/tmp/abtree_nohead"
    if os.path.exists(tmp):
        shutil.rmtree(tmp)
    os.makedirs(tmp)
    sh(f"cd {ROOT} && tar -cf - cfd-demo2_amd/csrc include __graft_entry__.py | tar -x -C {tmp}", shell=True)
    sh(f"git -C {ROOT} diff 0b05cfe^ 0b05cfe -- cfd-demo2_amd/csrc/hip/kernels.hip | patch -R -p1 -d {tmp}",
       shell=True)
    os.makedirs(os.path.join(tmp, "cfd-demo2_amd", "cfd2_amd", "_lib"), exist_ok=True)
    sh([sys.executable, "-c", "import __graft_entry__ as g; g.build_product(force=True)"], cwd=tmp)
    shutil.copy(os.path.join(tmp, "cfd-demo2_amd", "cfd2_amd", "_lib", "libcfd2_amd.so"),
                os.path.join(AB, "libcfd2_amd_nohead.so"))


for name in sys.argv[1:] or ["r04", "nokpre", "nohead"]:
    globals()[name]()
