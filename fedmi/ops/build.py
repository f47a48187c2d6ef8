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
import contextlib
import fcntl
import glob
import hashlib
import os
import re
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


def _headers() -> list:
    return sorted(glob.glob(os.path.join(CSRC, "*.h")) + glob.glob(os.path.join(CSRC, "*.inc")))


def source_digest() -> str:
    """Digest of every source and header the extension is built from (+ the target arch).
    It is compiled INTO the extension (``SRC_DIGEST``, and a marker string found by
    :func:`so_digest` without loading the library), so a binary can be matched to the tree it
    runs from wherever it travels -- the ``_build`` stamp does not go to the GPU box."""
    h = hashlib.sha256()
    for p in sorted(_sources() + _headers()):
        h.update(os.path.basename(p).encode())
        with open(p, "rb") as f:
            h.update(f.read())
    h.update(ARCH.encode())
    return h.hexdigest()[:16]


_MARKER = b"FEDMI_SRC_DIGEST:"


def so_digest(path: str = TARGET):
    """The source digest compiled into the extension at ``path`` (``None``: no file, or a
    binary built before digests were embedded).  Reads the file; never loads it."""
    try:
        with open(path, "rb") as f:
            data = f.read()
    except OSError:
        return None
    m = re.search(re.escape(_MARKER) + rb"([0-9a-f]{16})", data)
    return m.group(1).decode() if m else None


def build_digest() -> str:
    """What a build of this tree with the current ``FEDMI_HIPCC_FLAGS`` embeds: the source
    digest, or (experiment flags set) a digest of it and the flags, so a variant build is
    never taken for the plain one."""
    flags = os.environ.get("FEDMI_HIPCC_FLAGS", "").strip()
    if not flags:
        return source_digest()
    return hashlib.sha256((source_digest() + flags).encode()).hexdigest()[:16]


@contextlib.contextmanager
def _build_lock():
    """Exclusive across processes: N ranks that find the extension missing or stale at once
    build it one after another (the later ones then see a fresh binary and return)."""
    os.makedirs(BUILD, exist_ok=True)
    with open(os.path.join(BUILD, "lock"), "w") as f:
        fcntl.flock(f, fcntl.LOCK_EX)
        try:
            yield
        finally:
            fcntl.flock(f, fcntl.LOCK_UN)


def _compile(src: str, digest: str) -> str:
    obj = os.path.join(BUILD, os.path.basename(src) + ".o")
    extra = os.environ.get("FEDMI_HIPCC_FLAGS", "").split()  # experiments, e.g. -DFL_THREADS=1024
    cmd = ["hipcc", "-c", "-fPIC", "-O3", "-std=c++17", f"--offload-arch={ARCH}", *extra,
           f'-DFEDMI_SRC_DIGEST="{digest}"', "-I" + CSRC, *_pybind_includes(), src, "-o", obj]
    if src.endswith(".cpp"):
        cmd[1:1] = ["-x", "hip"]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"compile failed: {' '.join(cmd)}\n{r.stdout}\n{r.stderr}")
    return obj


def is_fresh() -> bool:
    """The in-tree extension exists and was built from the sources in this tree."""
    return so_digest(TARGET) == build_digest()


def build(force: bool = False, jobs: int = 8, verbose: bool = False) -> str:
    with _build_lock():
        return _build_locked(force, jobs, verbose)


def _build_locked(force: bool, jobs: int, verbose: bool) -> str:
    srcs = _sources()
    digest = build_digest()
    if not force and so_digest(TARGET) == digest:
        return TARGET
    os.makedirs(BUILD, exist_ok=True)
    with ThreadPoolExecutor(max_workers=max(1, min(jobs, len(srcs)))) as ex:
        objs = list(ex.map(lambda p: _compile(p, digest), srcs))
    tlib = _torch_lib()
    tmp = TARGET + f".tmp{os.getpid()}"
    link = ["g++", "-shared", "-o", tmp, *objs, f"-L{tlib}", "-lamdhip64", "-lrccl",
            f"-Wl,-rpath,{tlib}", "-Wl,--no-as-needed"]
    r = subprocess.run(link, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"link failed: {' '.join(link)}\n{r.stdout}\n{r.stderr}")
    os.replace(tmp, TARGET)  # atomic: a process mapping the old file keeps its copy
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
