"""In-tree build of libstochquant.so and tauhost.o for gfx950 (hipcc, no cmake).

    python -m stochquant_amd.build            # build if sources changed
    python -m stochquant_amd.build --force

Outputs (git-ignored, shipped to the GPU box with the working tree):
    stochquant_amd/lib/libstochquant.so
    stochquant_amd/bin/tauhost.o          (also linked as ./tauhost.o at the repo root,
                                           where taumain.py expects it)
"""
import argparse
import concurrent.futures as cf
import hashlib
import os
import shutil
import subprocess
import sys

PKG = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(PKG)
CSRC = os.path.join(PKG, "csrc")
OBJ = os.path.join(PKG, "_obj")
LIBDIR = os.path.join(PKG, "lib")
BINDIR = os.path.join(PKG, "bin")
LIB = os.path.join(LIBDIR, "libstochquant.so")
TAUHOST = os.path.join(BINDIR, "tauhost.o")
ROCM = os.environ.get("ROCM_PATH", "/opt/rocm")
HIPCC = os.path.join(ROCM, "bin", "hipcc")
ARCH = os.environ.get("SQ_OFFLOAD_ARCH", "gfx950")

DEVICE_SOURCES = ["sq_phi4.hip", "sq_phi4_run.hip", "sq_qm1d.hip", "sq_qm1d_gs.hip", "sq_selftest.hip", "sq_p2p.hip", "sq_fields.hip"]
HOST_SOURCES = ["sq_api.cpp", "sq_io.cpp"]
HEADERS = ["sq_internal.h", "sq_rng.h", "sq_dpp.h", "sq_glibcf.h"]
INCLUDES = {"sq_phi4_run.hip": ["sq_phi4.hip"]}  # device sources that include another one
COMMON = ["-O3", "-fPIC", "-std=c++17", "-ffp-contract=off", "-fno-slp-vectorize", "-Wall",
          "-Wno-unused-function"]


def _digest(paths, extra):
    h = hashlib.sha256()
    for p in paths:
        with open(p, "rb") as fh:
            h.update(fh.read())
    h.update(" ".join(extra).encode())
    return h.hexdigest()


def build_id(objs):
    """"phi4:<h> lib:<h>": sha256 (16 hex) of the φ⁴ kernels' object, and of every object in link order."""
    def h(paths):
        d = hashlib.sha256()
        for p in paths:
            with open(p, "rb") as fh:
                d.update(fh.read())
        return d.hexdigest()[:16]
    phi4 = [o for o in objs if os.path.basename(o) == "sq_phi4.hip.o"]
    return f"phi4:{h(phi4)} lib:{h(objs)}"


def _run(cmd):
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError("build failed:\n" + " ".join(cmd) + "\n" + r.stdout + r.stderr)
    return r


def build(force=False, verbose=False):
    """Compile every HIP translation unit for gfx950 and link the library + executable."""
    os.makedirs(OBJ, exist_ok=True)
    os.makedirs(LIBDIR, exist_ok=True)
    os.makedirs(BINDIR, exist_ok=True)
    hdrs = [os.path.join(CSRC, h) for h in HEADERS] + [os.path.join(ROOT, "include", "stochquant.h")]
    jobs = []
    for src in DEVICE_SOURCES + HOST_SOURCES:
        s = os.path.join(CSRC, src)
        o = os.path.join(OBJ, src + ".o")
        flags = COMMON + [f"--offload-arch={ARCH}", "-x", "hip"]
        stamp = o + ".sha"
        dig = _digest([s] + [os.path.join(CSRC, d) for d in INCLUDES.get(src, [])] + hdrs, flags)
        if not force and os.path.exists(o) and os.path.exists(stamp) and open(stamp).read() == dig:
            continue
        jobs.append(([HIPCC] + flags + ["-c", s, "-o", o], stamp, dig))
    with cf.ThreadPoolExecutor(max_workers=min(8, os.cpu_count() or 4)) as ex:
        for (cmd, stamp, dig), _ in zip(jobs, ex.map(lambda j: _run(j[0]), jobs)):
            with open(stamp, "w") as fh:
                fh.write(dig)
            if verbose:
                print(" ".join(cmd))
    objs = [os.path.join(OBJ, s + ".o") for s in DEVICE_SOURCES + HOST_SOURCES]
    bid = build_id(objs)
    bid_obj = os.path.join(OBJ, "sq_build_id.cpp.o")
    bid_stamp = bid_obj + ".sha"
    if jobs or force or not os.path.exists(bid_obj) or not os.path.exists(bid_stamp) or \
            open(bid_stamp).read() != bid:
        # the identity of the objects just built, compiled into the library (sq_build_id)
        _run([HIPCC] + COMMON + ["-x", "c++", f'-DSQ_BUILD_ID="{bid}"', "-c",
                                 os.path.join(CSRC, "sq_build_id.cpp"), "-o", bid_obj])
        with open(bid_stamp, "w") as fh:
            fh.write(bid)
        jobs.append(None)
    if jobs or force or not os.path.exists(LIB):
        _run([HIPCC, f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", LIB] + objs + [bid_obj]
             + [f"-L{ROCM}/lib", "-lrccl", f"-Wl,-rpath,{ROCM}/lib"])
    th_src = os.path.join(CSRC, "tauhost.cpp")
    if jobs or force or not os.path.exists(TAUHOST) or \
            os.path.getmtime(th_src) > os.path.getmtime(TAUHOST):
        _run(["g++", "-O2", "-std=c++17", "-Wall", "-o", TAUHOST, th_src,
              f"-L{LIBDIR}", "-lstochquant", "-Wl,-rpath,$ORIGIN/../lib", f"-Wl,-rpath,{ROCM}/lib", "-lm"])
    root_link = os.path.join(ROOT, "tauhost.o")
    try:
        if os.path.islink(root_link) or os.path.exists(root_link):
            os.remove(root_link)
        os.symlink(os.path.relpath(TAUHOST, ROOT), root_link)
    except OSError:
        shutil.copy2(TAUHOST, root_link)
    return LIB


def build_oracle(verbose=False):
    """Build oracle/liboracle.so (test infrastructure) with its Makefile."""
    odir = os.path.join(ROOT, "oracle")
    r = subprocess.run(["make", "-C", odir, "-j4"], capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError("oracle build failed:\n" + r.stdout + r.stderr)
    if verbose:
        print(r.stdout)
    return os.path.join(odir, "liboracle.so")


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--force", action="store_true")
    ap.add_argument("-v", "--verbose", action="store_true")
    a = ap.parse_args(argv)
    print(build(force=a.force, verbose=a.verbose))
    print(build_oracle(verbose=a.verbose))


if __name__ == "__main__":
    sys.exit(main())
