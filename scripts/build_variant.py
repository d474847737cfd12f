"""Build a variant of the gfx950 kernel library with extra compile flags (tuning A/B).

    python scripts/build_variant.py NAME [-DMACRO=V ...]

-> mpi_cuda_largescaleknn_amd/lib/exp/liblsknn_hip_NAME.so, loaded by any script with
LSKNN_HIP_LIB=<that path> (knn_engine and the tests then run the variant).
"""
import concurrent.futures as cf
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from mpi_cuda_largescaleknn_amd import _build as B  # noqa: E402


def main():
    name, defs = sys.argv[1], sys.argv[2:]
    out_dir = os.path.join(B.LIB_DIR, "exp")
    obj_dir = os.path.join(out_dir, "obj_" + name)
    os.makedirs(obj_dir, exist_ok=True)
    srcs = B._sources("hip", "hip")

    def one(src):
        obj = os.path.join(obj_dir, os.path.basename(src) + ".o")
        B._run([B._hipcc(), *B.HIP_FLAGS, *B.FILE_FLAGS.get(os.path.basename(src), []), *defs, "-c", src,
                "-o", obj])
        return obj

    with cf.ThreadPoolExecutor(8) as ex:
        objs = list(ex.map(one, srcs))
    lib = os.path.join(out_dir, f"liblsknn_hip_{name}.so")
    B._run([B._hipcc(), f"--offload-arch={B.GPU_ARCH}", "-shared", "-fPIC", "-o", lib, *objs])
    print(lib)


if __name__ == "__main__":
    main()
