"""fv_build.py -- build a diagnostic variant of libgwa for the gfx950 flag-form study:
the -m sf children loop of `SfLane::sfStepT` (sf_core.h) rewritten from its early `return end` into a
loop-carried `ok` flag, optionally with instrumentation, recompiled for the one search instance the
400-bp test runs (QW 16, R 32) with extra compiler flags, and linked with the other objects of the
in-tree build (genome-weaver-align_amd/build/).  Tools only; the product keeps the early return.

  python tools/fv_build.py NAME MODE [compiler flags ...]   -> genome-weaver-align_amd/libgwa_fv_NAME.so
  MODE: flag     the flag form
        vflag    the flag form with the flag pinned to a VGPR each iteration (empty asm)
        flagdbg  the flag form + device counters (children taken) read by gwa_dbg_read
        retdbg   the early-return form + the same counters
  e.g.  python tools/fv_build.py b57516 flag -mllvm -opt-bisect-limit=57516
Then: bash tools/fv_run.sh NAME ... on the GPU box, or GWA_LIB=libgwa_fv_NAME.so tools/fv_isolate.py.
"""
import glob
import os
import shutil
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(REPO, "genome-weaver-align_amd")

LOOP_RET = """    for (int ch = 0; ch < 4; ++ch) {  // ACGT.exceptN
      const uint64_t l = ix.C[ch] + lo[ch], u = ix.C[ch] + hi[ch];
      if (l < u && !child(c, ch, (uint32_t)l, (uint32_t)u)) return end;
    }
    return 1;"""
LOOP_FLAG = """    int ok = 1;
    for (int ch = 0; ch < 4; ++ch) {  // ACGT.exceptN
      const uint64_t l = ix.C[ch] + lo[ch], u = ix.C[ch] + hi[ch];
      if (ok && l < u && !child(c, ch, (uint32_t)l, (uint32_t)u)) ok = 0;%s
    }
    return ok ? 1 : end;"""
PIN = """
      ok = pinv(ok);"""
CHILD = """    if (!B::stairOk()) return false;  // c.nextState(..., getStairCaseFilter(m)) (:282)
"""
COUNT = """#if defined(__HIP_DEVICE_COMPILE__)
    if (pinv(lb) >= pinv(ub)) atomicAdd(&gwaDbg[0], 1u);  // children with an empty interval
    atomicAdd(&gwaDbg[1], 1u);                             // children taken
#endif
"""
READER = """
extern "C" int gwa_dbg_read(unsigned *out) {  // diagnostic variant: read and clear gwaDbg
  if (hipMemcpyFromSymbol(out, HIP_SYMBOL(gwaDbg), 4 * sizeof(unsigned)) != hipSuccess) return -1;
  const unsigned z[4] = {0, 0, 0, 0};
  return hipMemcpyToSymbol(HIP_SYMBOL(gwaDbg), z, sizeof(z)) == hipSuccess ? 0 : -1;
}
"""


def main():
    name, mode, flags = sys.argv[1], sys.argv[2], sys.argv[3:]
    d = "/tmp/gwa_fv_" + name
    shutil.rmtree(d, ignore_errors=True)
    os.makedirs(os.path.join(d, "include"))
    shutil.copytree(os.path.join(PKG, "csrc"), os.path.join(d, "pkg", "csrc"))
    shutil.copy(os.path.join(REPO, "include", "gwa.h"), os.path.join(d, "include"))
    src = os.path.join(d, "pkg", "csrc")
    s = open(os.path.join(src, "sf_core.h")).read()
    assert s.count(LOOP_RET) == 1 and s.count(CHILD) == 1
    if mode in ("flag", "vflag", "flagdbg"):
        s = s.replace(LOOP_RET, LOOP_FLAG % (PIN if mode == "vflag" else ""))
    if mode in ("flagdbg", "retdbg"):
        s = s.replace('#include "bsf_core.h"\n', '#include "bsf_core.h"\n__device__ unsigned gwaDbg[4];\n', 1)
        s = s.replace(CHILD, COUNT + CHILD)
        with open(os.path.join(src, "search_inst.hip"), "a") as f:
            f.write(READER)
    open(os.path.join(src, "sf_core.h"), "w").write(s)
    obj = os.path.join(d, "search_q16_r32.o")
    subprocess.check_call(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC",
                           "-Wno-unused-function", "-Wno-sign-compare"] + flags +
                          ["-DGWA_QW=16", "-DGWA_R=32", "-c", "csrc/search_inst.hip", "-o", obj],
                          cwd=os.path.join(d, "pkg"))
    objs = [o for o in sorted(glob.glob(os.path.join(PKG, "build", "*.o"))) if not o.endswith("search_q16_r32.o")]
    out = os.path.join(PKG, "libgwa_fv_%s.so" % name)
    subprocess.check_call(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-shared", "-fPIC", "-fopenmp", "-o", out]
                          + objs + [obj, "-lz"])
    print("built", out)


if __name__ == "__main__":
    main()
