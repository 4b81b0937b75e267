"""Build an experiment variant of liblspcg_hip.so: one translation unit recompiled with extra
compiler flags, linked with the in-tree objects of the others (build/lspcg/*.o, from a normal
build first).  Measurement only: load it with LSPCG_LIB=<path> (tools/gnn_ab.py).

    python tools/build_variant.py exp/liblspcg_gs.so lspcg_gnn.hip -DLSPCG_GELU_SCALAR
    python tools/build_variant.py tools/_variants/libx.so lspcg_pcg.hip,lspcg_core.hip -DX=1  (several units)
"""
import subprocess
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
from learningsparsepreconditioner4gpu_amd import _build as B


def main():
    out, srcs, flags = Path(sys.argv[1]), sys.argv[2].split(","), sys.argv[3:]
    B.build(verbose=False)
    out.parent.mkdir(parents=True, exist_ok=True)
    objs_v = {}
    for src in srcs:
        obj = out.with_name(out.stem + "_" + Path(src).stem + ".o")
        cmd = B._cmd(src, B.tree_hash())
        cmd = cmd[:-2] + list(flags) + ["-o", str(obj)]
        subprocess.run(cmd, check=True)
        objs_v[src] = obj
    objs = [str(objs_v[s]) if s in objs_v else str(B._obj(s)) for s in B.SOURCES]
    subprocess.run([B.hipcc(), "-shared", f"--offload-arch={B.ARCH}", *objs, "-o", str(out)], check=True)
    for obj in objs_v.values():
        obj.unlink()
    print(out)


if __name__ == "__main__":
    main()
