"""In-tree build of the native extension ``fedmi/ops/_fedmi_hip*.so`` for gfx950.

Every ``*.hip`` / ``*.cpp`` under ``fedmi/ops/csrc`` is compiled with ``hipcc
--offload-arch=gfx950`` (in parallel), then linked with g++ against the HIP runtime and
RCCL that *torch* ships (``torch/lib``): loading a second HIP runtime into the same
process would give the extension its own device context, so the extension must resolve
``libamdhip64.so`` / ``librccl.so`` to the copies torch already loaded.

Usage: ``python -m fedmi.ops.build [--force] [-j N]``.
"""
from __future__ import annotations

import argparse
import glob
import hashlib
import os
import subprocess
import sys
import sysconfig
from concurrent.futures import ThreadPoolExecutor

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "csrc")
BUILD = os.path.join(HERE, "_build")
ARCH = os.environ.get("FEDMI_ARCH", "gfx950")
EXT_SUFFIX = sysconfig.get_config_var("EXT_SUFFIX") or ".so"
TARGET = os.path.join(HERE, "_fedmi_hip" + EXT_SUFFIX)


def _torch_lib() -> str:
    import importlib.util
    spec = importlib.util.find_spec("torch")
    if spec is None or spec.origin is None:
        raise RuntimeError("torch not importable; it provides the HIP runtime the extension links to")
    return os.path.join(os.path.dirname(spec.origin), "lib")


def _pybind_includes() -> list:
    import pybind11
    return ["-I" + pybind11.get_include(), "-I" + sysconfig.get_paths()["include"]]


def _sources() -> list:
    return sorted(glob.glob(os.path.join(CSRC, "*.hip")) + glob.glob(os.path.join(CSRC, "*.cpp")))


def _digest(paths) -> str:
    h = hashlib.sha256()
    for p in sorted(paths):
        with open(p, "rb") as f:
            h.update(f.read())
    h.update(ARCH.encode())
    h.update(os.environ.get("FEDMI_HIPCC_FLAGS", "").encode())
    return h.hexdigest()[:16]


def _compile(src: str) -> str:
    obj = os.path.join(BUILD, os.path.basename(src) + ".o")
    extra = os.environ.get("FEDMI_HIPCC_FLAGS", "").split()  # experiments, e.g. -DFL_THREADS=1024
    cmd = ["hipcc", "-c", "-fPIC", "-O3", "-std=c++17", f"--offload-arch={ARCH}", *extra,
           "-I" + CSRC, *_pybind_includes(), src, "-o", obj]
    if src.endswith(".cpp"):
        cmd[1:1] = ["-x", "hip"]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"compile failed: {' '.join(cmd)}\n{r.stdout}\n{r.stderr}")
    return obj


def build(force: bool = False, jobs: int = 8, verbose: bool = False) -> str:
    srcs = _sources()
    headers = glob.glob(os.path.join(CSRC, "*.h")) + glob.glob(os.path.join(CSRC, "*.inc"))
    stamp = os.path.join(BUILD, "stamp")
    digest = _digest(srcs + headers)
    if not force and os.path.isfile(TARGET) and os.path.isfile(stamp):
        with open(stamp) as f:
            if f.read().strip() == digest:
                return TARGET
    os.makedirs(BUILD, exist_ok=True)
    with ThreadPoolExecutor(max_workers=max(1, min(jobs, len(srcs)))) as ex:
        objs = list(ex.map(_compile, srcs))
    tlib = _torch_lib()
    link = ["g++", "-shared", "-o", TARGET, *objs, f"-L{tlib}", "-lamdhip64", "-lrccl",
            f"-Wl,-rpath,{tlib}", "-Wl,--no-as-needed"]
    r = subprocess.run(link, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"link failed: {' '.join(link)}\n{r.stdout}\n{r.stderr}")
    with open(stamp, "w") as f:
        f.write(digest)
    if verbose:
        print(f"built {TARGET}")
    return TARGET


def main(argv=None) -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--force", action="store_true")
    ap.add_argument("-j", "--jobs", type=int, default=8)
    a = ap.parse_args(argv)
    build(force=a.force, jobs=a.jobs, verbose=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
