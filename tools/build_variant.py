#!/usr/bin/env python3
"""Build a variant of libngrtd.so with extra compiler flags (A/B runs, tools/gpu_ab_libs.sh):

    python tools/build_variant.py NAME -DNGRTD_NO_FMA_K [...]   -> noblegas_rtd_mcmc_amd/libngrtd_NAME.so

Both translation units get the flags; run the product code against it with
NGRTD_LIB=$PWD/noblegas_rtd_mcmc_amd/libngrtd_NAME.so."""
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def main():
    import __graft_entry__ as g
    name, flags = sys.argv[1], sys.argv[2:]
    out = os.path.join(REPO, "noblegas_rtd_mcmc_amd", "libngrtd_%s.so" % name)
    objs, procs = [], []
    for src in g._sources():
        obj = "%s.%s.o" % (src, name)
        cmd = ["hipcc"] + g.HIPCC_FLAGS + g.EXTRA_FLAGS.get(os.path.basename(src), []) + flags + ["-c", "-o", obj, src]
        procs.append(subprocess.Popen(cmd))
        objs.append(obj)
    if any(p.wait() for p in procs):
        sys.exit("compile failed")
    subprocess.run(["hipcc", "--offload-arch=gfx950", "-shared", "-fPIC", "-o", out] + objs + ["-ldl"], check=True)
    for o in objs:
        os.remove(o)
    print(out)


if __name__ == "__main__":
    main()
