"""Build helpers: compile libtgsim.so for gfx950 in-tree and the CPU oracle.

The product library is built with ``hipcc --offload-arch=gfx950`` straight into
``testground_amd/libtgsim.so`` so that it travels to the GPU box with the repository snapshot.
"""
from __future__ import annotations

import os
import subprocess
from pathlib import Path

PKG = Path(__file__).resolve().parent
ROOT = PKG.parent
CSRC = PKG / "csrc"
LIB = PKG / "libtgsim.so"
SOURCES = [CSRC / "tgsim_kernels.hip", CSRC / "tgsim_engine.cpp", CSRC / "tgsim_bridge.cpp", CSRC / "tgsim_comm.cpp"]
HEADERS = [CSRC / "tgsim_internal.h", CSRC / "tgsim_launch.h", ROOT / "include" / "tgsim.h"]
ORACLE_DIR = ROOT / "oracle"
ORACLE_LIB = ORACLE_DIR / "build" / "libtgoracle.so"

HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
ARCH = os.environ.get("PYTORCH_ROCM_ARCH", "gfx950")


def _stale(target: Path, deps) -> bool:
    if not target.exists():
        return True
    t = target.stat().st_mtime
    return any(Path(d).stat().st_mtime > t for d in deps)


PROF_LIB = PKG / "libtgsim_prof.so"
CHECK_LIB = PKG / "libtgsim_check.so"


def build_engine(force: bool = False, verbose: bool = False, profile: bool = False, check: bool = False) -> Path:
    """Compiles the HIP engine (kernels + host runtime) into libtgsim.so.  profile=True builds the
    diagnostic variant libtgsim_prof.so (k_sim cycle counters in the stamp slots; scripts only);
    check=True the invariant-checking variant libtgsim_check.so (-DTGSIM_CHECK: queue invariants and
    the cross-lane exec-mask guards; loaded by TGSIM_LIB=... for scripts/check_build.sh only)."""
    lib = PROF_LIB if profile else CHECK_LIB if check else LIB
    if not force and not _stale(lib, SOURCES + HEADERS):
        return lib
    objs = []
    build_dir = PKG / ("build_prof" if profile else "build_check" if check else "build")
    build_dir.mkdir(exist_ok=True)
    for src in SOURCES:
        obj = build_dir / (src.stem + ".o")
        # the AMDGPU register-pressure trackers in the scheduler: 40 % fewer SGPR spills in k_sim
        # and 1.2 % off its time (A/B on the GPU)
        # (no promotion of private arrays to LDS: it gives the scatter kernels 0.75-12 KiB of LDS per
        # workgroup for a record copy; sub-capacity storm 1.31 against 1.17 G pkt/s without it,
        # the 1M-peer gossip unchanged, profiles/r05/ab/twelfth_*)
        dev = ["-mllvm", "-amdgpu-use-amdgpu-trackers=1", "-mllvm", "-disable-promote-alloca-to-lds"] \
            if src.suffix == ".hip" else []
        cmd = [HIPCC, f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC", "-Wall", *dev,
               "-Wno-unused-result", *(["-DTGSIM_PROFILE"] if profile else []),
               *(["-DTGSIM_CHECK"] if check else []), "-c", str(src), "-o", str(obj)]
        if verbose:
            print(" ".join(cmd))
        subprocess.run(cmd, check=True)
        objs.append(str(obj))
    cmd = [HIPCC, f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", str(lib), *objs]
    if verbose:
        print(" ".join(cmd))
    subprocess.run(cmd, check=True)
    return lib


def build_oracle(force: bool = False) -> Path:
    """Compiles the CPU golden model (test infrastructure).  TGORACLE_LIB names another build of
    it (the sanitizer build of scripts/sanitize.sh) to load instead."""
    if os.environ.get("TGORACLE_LIB"):
        return Path(os.environ["TGORACLE_LIB"])
    if force or _stale(ORACLE_LIB, [ORACLE_DIR / "tgoracle.c", ORACLE_DIR / "tgoracle.h", ROOT / "include" / "tgsim.h"]):
        subprocess.run(["make", "-C", str(ORACLE_DIR), "-B" if force else "all"], check=True,
                       stdout=subprocess.DEVNULL)
    return ORACLE_LIB


MOCK_DIR = ROOT / "tests" / "mockrccl"
MOCK_COMM_LIB = MOCK_DIR / "libtgsim_mockcomm.so"


def build_engine_mockcomm(force: bool = False) -> Path:
    """TEST build of the engine for tests/test_gpu_multirank.py: the product's kernel, engine and
    bridge objects, tgsim_comm.cpp recompiled with -DTGSIM_COMM_TEST_TRANSPORT and the ranks-as-threads
    transport of tests/mockrccl linked in (RCCL refuses two ranks on one GPU).  Lives under tests/;
    libtgsim.so never contains it."""
    prod = build_engine()
    srcs = [CSRC / "tgsim_comm.cpp", MOCK_DIR / "mock_rccl.cpp"]
    if not force and not _stale(MOCK_COMM_LIB, srcs + HEADERS + [prod]):
        return MOCK_COMM_LIB
    objs = [str(PKG / "build" / (s.stem + ".o")) for s in SOURCES if s.stem != "tgsim_comm"]
    for src in srcs:
        obj = MOCK_DIR / (src.stem + ".o")
        subprocess.run([HIPCC, f"--offload-arch={ARCH}", "-O2", "-std=c++17", "-fPIC", "-Wall", "-Wno-unused-result",
                        "-DTGSIM_COMM_TEST_TRANSPORT", "-c", str(src), "-o", str(obj)], check=True)
        objs.append(str(obj))
    subprocess.run([HIPCC, f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", str(MOCK_COMM_LIB), *objs], check=True)
    return MOCK_COMM_LIB


def build_engine_host_asan() -> Path:
    """libtgsim built with AddressSanitizer + UBSan on its HOST code only (-Xarch_host; GPU code is
    never sanitized on this pool): the CPU tests of the C ABI (tests/test_abi.py) load it."""
    lib = PKG / "build_asan" / "libtgsim_asan.so"
    lib.parent.mkdir(exist_ok=True)
    san = ["-Xarch_host", "-fsanitize=address", "-Xarch_host", "-fsanitize=undefined",
           "-Xarch_host", "-fno-sanitize-recover=all", "-Xarch_host", "-fno-omit-frame-pointer"]
    objs = []
    for src in SOURCES:
        obj = lib.parent / (src.stem + ".o")
        subprocess.run([HIPCC, f"--offload-arch={ARCH}", "-O1", "-g", "-std=c++17", "-fPIC", *san, "-c", str(src),
                        "-o", str(obj)], check=True)
        objs.append(str(obj))
    subprocess.run([HIPCC, f"--offload-arch={ARCH}", "-shared", "-fPIC", *san, "-o", str(lib), *objs], check=True)
    return lib


if __name__ == "__main__":
    build_engine(force=True, verbose=True)
    build_oracle(force=True)
