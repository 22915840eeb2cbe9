"""Per-phase cycle timing of step_v2 <DEFER> and fear_v2 (a measurement experiment, run on the box).

Patches a COPY of csrc/gridenv.hip with s_memtime stamps (clock64) taken by lane 0 of each block
at the phase boundaries, builds it next to the copy, runs C3 steps through it and prints the mean
/ p50 / p90 cycles of each phase over all blocks of one step.  The shipped library is untouched.
Usage (on the GPU box):  python tools/phase_timing.py [scenario] [envs]
"""
import ctypes as C
import os
import subprocess
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(ROOT, "marl-responsible-nav_amd", "csrc", "gridenv.hip")
OUT = os.path.join(ROOT, "gpurun_out", "phase")

STAMP = "if (threadIdx.x == 0 && blockIdx.x < 65536u) gw_phase_clk[blockIdx.x][{slot}] = clock64();\n"


def patch(src: str) -> str:
    def ins(s, anchor, text, after=True, count=1):
        assert s.count(anchor) == count, (anchor, s.count(anchor))
        return s.replace(anchor, anchor + text if after else text + anchor)

    src = ins(src, "namespace gw {\n", "__device__ unsigned long long gw_phase_clk[65536][8];\n"
              "__device__ unsigned long long gw_fear_clk[65536][8];\n")
    # step_v2: start / tables+state in LDS / actions / world update / finish / end
    a = src.index("__device__ __forceinline__ void step_v2_block(")
    b1 = src.index("template <int N, int KMAX, bool FEAR, bool OBS, bool DEFER = false>\n"
                   "__global__ void __launch_bounds__(128) step_v2(Params p) {")
    b = src.index("__global__ void __launch_bounds__(128) fear_v2(Params p) {")
    step, mid, rest = src[a:b1], src[b1:b], src[b:]
    step = ins(step, "    const int tid = threadIdx.x;\n", "    " + STAMP.format(slot=0))
    step = ins(step, "    const CtabOk okv{ctab};\n", "    " + STAMP.format(slot=1))
    step = ins(step, "            select_actions_v2<N>(p, e, es, ctab, cdf_s, act);\n#pragma unroll\n            for (int n = 0; n < N; ++n) {\n                pos[n] = es.pos[n];\n                mdr[n] = (int)((ctab[pos[n]] >> CT_MDR) & 0xFu);\n            }\n",
               "            " + STAMP.format(slot=2))
    step = ins(step, "            simulate<N, true>(w, okv, K, apple, caught, fin);\n            double fear[MAXN];\n",
               "            " + STAMP.format(slot=3))
    step = ins(step, "            finish_env<N, DEFER>(p, e, es, act, mdr, fear, w.crash, w.restr, fin, caught, ct, oi, ctab);\n",
               "            " + STAMP.format(slot=4))
    step = ins(step, "                store_desc<N>(p, e, oi);\n            }\n        }\n    }\n", "    " + STAMP.format(slot=5))
    step = ins(step, "    block_stats<T>(p, ct, sh.red, tid, p.stats_row0 + e0 / BE);\n", "    " + STAMP.format(slot=6))
    fstamp = STAMP.replace("gw_phase_clk", "gw_fear_clk")
    fear_end = rest.index("\n}\n") + 3
    fear, tail = rest[:fear_end], rest[fear_end:]
    fear = ins(fear, "    const int tid = threadIdx.x;\n", "    " + fstamp.format(slot=0))
    fear = ins(fear, "    const CtabOk okv{ctab};\n", "    " + fstamp.format(slot=1))
    fear = ins(fear, "    // ---- B ----\n", "    " + fstamp.format(slot=2))
    fear = ins(fear, "    // ---- C ----\n", "    " + fstamp.format(slot=3))
    fear = ins(fear, "        ct.v[5] = np_sum_small(shaped, K);\n    }\n", "    " + fstamp.format(slot=4))
    fear = ins(fear, "    block_stats<T>(p, ct, sh.red, tid, p.stats_row0 + e0 / BE);\n", "    " + fstamp.format(slot=5))
    fear = ins(fear, "        fear_plan<N, KMAX>(p, sh, tid, pos, act, 0);\n", "        " + fstamp.format(slot=6), after=False)
    src = src[:a] + step + mid + fear + tail
    src += ('\nextern "C" int gw_phase_read(unsigned long long *step, unsigned long long *fear, int n) {\n'
            '    if (hipMemcpyFromSymbol(step, HIP_SYMBOL(gw::gw_phase_clk), sizeof(unsigned long long) * 8 * n) != hipSuccess) return -1;\n'
            '    return hipMemcpyFromSymbol(fear, HIP_SYMBOL(gw::gw_fear_clk), sizeof(unsigned long long) * 8 * n) == hipSuccess ? 0 : -1;\n}\n')
    return src


def main():
    scen = sys.argv[1] if len(sys.argv) > 1 else "grid32"
    E = int(sys.argv[2]) if len(sys.argv) > 2 else 65536
    fear = bool(int(sys.argv[3])) if len(sys.argv) > 3 else True
    os.environ.setdefault("GW_KERNEL", "defer")
    os.makedirs(OUT, exist_ok=True)
    with open(SRC) as f:
        src = patch(f.read())
    hip = os.path.join(OUT, "gridenv_phase.hip")
    with open(hip, "w") as f:
        f.write(src)
    sys.path.insert(0, os.path.join(ROOT, "marl-responsible-nav_amd"))
    import torch  # noqa: F401  (shared HIP runtime, before the library loads)
    from marlnav import _lib
    lib_path = os.path.join(OUT, "libgridenv_phase.so")
    cmd = [_lib.HIPCC, *_lib.HIPCC_FLAGS, f"-I{_lib.INCLUDE}", hip, *_lib.HIP_SOURCES[1:], "-o", lib_path]
    subprocess.run(cmd, check=True)
    _lib.LIB_PATH = lib_path
    _lib.needs_build = lambda: False
    from marlnav.vec_env import VecGridEnv
    env = VecGridEnv(scen, num_envs=E, fear=fear, fear_weight=-5.0, stats=True)
    env.reset()
    for _ in range(30):
        env.step()
    torch.cuda.synchronize()
    lib = env.lib
    n = 65536
    st = np.zeros((n, 8), np.uint64)
    fe = np.zeros((n, 8), np.uint64)
    lib.gw_phase_read.argtypes = [C.c_void_p, C.c_void_p, C.c_int]
    assert lib.gw_phase_read(st.ctypes.data, fe.ctypes.data, n) == 0
    for name, arr, labels in (("step_v2<DEFER>", st, ["fill+state", "actions", "simulate", "finish_env", "desc", "stats"]),
                              ("fear_v2", fe, ["fill+rec", "plan(A)", "sims(B)", "resp(C)", "stats"])):
        used = arr[:, 0] != 0
        if not used.any():
            continue
        a = arr[used].astype(np.int64)
        last = len(labels)
        print(f"{name}: {used.sum()} blocks; block span cycles mean {np.mean(a[:, last] - a[:, 0]):.0f}")
        for i, lab in enumerate(labels):
            d = a[:, i + 1] - a[:, i]
            print(f"  {lab:12s} mean {d.mean():8.0f}  p50 {np.percentile(d, 50):8.0f}  p90 {np.percentile(d, 90):8.0f}")
    a = fe[fe[:, 0] != 0].astype(np.int64)
    if len(a):
        print(f"  fear_v2 A split: decode {np.mean(a[:, 6] - a[:, 1]):.0f}  fear_plan+barrier {np.mean(a[:, 2] - a[:, 6]):.0f}")
    env.close()


if __name__ == "__main__":
    main()
