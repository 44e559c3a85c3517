"""Build libstochquant.so with a patched copy of one device source, for A/B runs
(SQ_LIB=<path> selects it at load time).

    python scripts/build_variant.py <patched source> <name> [replaced source, default sq_phi4.hip]
      -> stochquant_amd/lib/variants/libstochquant_<name>.so
"""
import os
import shutil
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from stochquant_amd import build  # noqa: E402


def main():
    src, name = sys.argv[1], sys.argv[2]
    which = sys.argv[3] if len(sys.argv) > 3 else "sq_phi4.hip"
    assert which in build.DEVICE_SOURCES, which
    build.build()
    tmp = os.path.join(ROOT, "stochquant_amd", "_obj", "variants", name)
    os.makedirs(tmp, exist_ok=True)
    dst_src = os.path.join(build.CSRC, "_variant_" + name + ".hip")
    shutil.copy(src, dst_src)
    try:
        obj = os.path.join(tmp, which + ".o")
        subprocess.run([build.HIPCC] + build.COMMON + [f"--offload-arch={build.ARCH}", "-x", "hip", "-c", dst_src,
                        "-o", obj], check=True)
    finally:
        os.remove(dst_src)
    objs = [obj] + [os.path.join(build.OBJ, s + ".o") for s in build.DEVICE_SOURCES + build.HOST_SOURCES
                    if s != which] + [os.path.join(build.OBJ, "sq_build_id.cpp.o")]  # the base build's identity
    out = os.path.join(build.LIBDIR, "variants", f"libstochquant_{name}.so")
    os.makedirs(os.path.dirname(out), exist_ok=True)
    subprocess.run([build.HIPCC, f"--offload-arch={build.ARCH}", "-shared", "-fPIC", "-o", out] + objs
                   + [f"-L{build.ROCM}/lib", "-lrccl", f"-Wl,-rpath,{build.ROCM}/lib"], check=True)
    print(out)


if __name__ == "__main__":
    main()
