"""ctypes binding of libgridenv.so (include/gridenv.h) and its in-tree build.

The library is built in-tree for gfx950 (``hipcc --offload-arch=gfx950``) so that the .so
travels with the repository snapshot.  torch must be imported before the library is loaded:
both then share torch's HIP runtime (same soname), and the device pointers / streams torch
hands out are valid for our kernels.  There is no CPU fallback: if the library cannot be
built or loaded, every entry point raises.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess
import threading

HERE = os.path.dirname(os.path.abspath(__file__))
PKG_ROOT = os.path.dirname(HERE)
REPO_ROOT = os.path.dirname(PKG_ROOT)
CSRC = os.path.join(PKG_ROOT, "csrc")
INCLUDE = os.path.join(REPO_ROOT, "include")
# MARLNAV_MEASURE=1: the measurement build (-DGW_MEASURE, csrc/measure.h: the kernels' A/B, probe
# and block-stamp switches read from the environment), a separate library and object cache; the
# release library (the product, the default) compiles those switches out
MEASURE = os.environ.get("MARLNAV_MEASURE", "0") == "1"
LIB_PATH = os.path.join(CSRC, "libgridenv_measure.so" if MEASURE else "libgridenv.so")
HIP_SOURCES = [os.path.join(CSRC, "gridenv.hip"), os.path.join(CSRC, "learner_ops.hip"),
               os.path.join(CSRC, "actor_ops.hip"), os.path.join(CSRC, "rollout_ops.hip"),
               os.path.join(CSRC, "maddpg_ops.hip"), os.path.join(CSRC, "patch_ops.hip")]
HEADERS = [os.path.join(INCLUDE, "gridenv.h"), os.path.join(INCLUDE, "learner_ops.h"),
           os.path.join(INCLUDE, "actor_ops.h"), os.path.join(INCLUDE, "rollout_ops.h")]
SOURCES = HIP_SOURCES + HEADERS + [os.path.join(CSRC, "patch_ops.h"), os.path.join(CSRC, "window_rows.h"), os.path.join(CSRC, "prof.h"),
                                   os.path.join(CSRC, "philox.h"), os.path.join(CSRC, "measure.h")]
OBJ_DIR = os.path.join(CSRC, "build_measure" if MEASURE else "build")
ARCH = os.environ.get("MARLNAV_OFFLOAD_ARCH", "gfx950")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")

HIPCC_FLAGS = ["-O3", f"--offload-arch={ARCH}", "-std=c++17", "-fPIC", "-shared",
               "-ffp-contract=off", "-fno-fast-math", "-Wall"] + (["-DGW_MEASURE"] if MEASURE else [])
COMPILE_FLAGS = [f for f in HIPCC_FLAGS if f != "-shared"]

GW_MAX_AGENTS = 8
_lock = threading.Lock()
_lib = None


class GwError(RuntimeError):
    pass


STAMP_PATH = LIB_PATH + ".sha256"


def source_hash() -> str:
    """Content hash of the sources + compile flags (mtimes change when the tree is copied)."""
    import hashlib
    h = hashlib.sha256(" ".join(HIPCC_FLAGS).encode())
    for src in SOURCES:
        with open(src, "rb") as f:
            h.update(f.read())
    return h.hexdigest()


def needs_build() -> bool:
    if not os.path.exists(LIB_PATH) or not os.path.exists(STAMP_PATH):
        return True
    with open(STAMP_PATH) as f:
        return f.read().strip() != source_hash()


def _deps(src: str) -> list:
    """src and the quoted #include files it pulls in (transitively) from csrc/ and include/."""
    import re
    seen, todo = [], [src]
    while todo:
        path = todo.pop()
        if path in seen:
            continue
        seen.append(path)
        with open(path) as f:
            for name in re.findall(r'^\s*#\s*include\s+"([^"]+)"', f.read(), re.M):
                for d in (os.path.dirname(path), INCLUDE, CSRC):
                    cand = os.path.join(d, name)
                    if os.path.exists(cand):
                        todo.append(cand)
                        break
    return seen


def _object(src: str, verbose: bool) -> str:
    """Compile one HIP source to csrc/build/<name>.<hash>.o (hash of the source, every header
    and the flags), reusing an existing object: only the changed translation units rebuild."""
    import hashlib
    h = hashlib.sha256(" ".join(COMPILE_FLAGS).encode())
    for path in _deps(src):
        with open(path, "rb") as f:
            h.update(f.read())
    name = os.path.splitext(os.path.basename(src))[0]
    obj = os.path.join(OBJ_DIR, f"{name}.{h.hexdigest()[:16]}.o")
    if os.path.exists(obj):
        return obj
    os.makedirs(OBJ_DIR, exist_ok=True)
    for old in os.listdir(OBJ_DIR):  # drop this source's stale objects
        if old.startswith(name + ".") and old.endswith(".o"):
            os.remove(os.path.join(OBJ_DIR, old))
    tmp = obj + f".tmp{os.getpid()}"
    cmd = [HIPCC, *COMPILE_FLAGS, f"-I{INCLUDE}", "-c", src, "-o", tmp]
    if verbose:
        print(" ".join(cmd), flush=True)
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise GwError(f"hipcc failed on {os.path.basename(src)} ({r.returncode}):\n{r.stderr[-4000:]}")
    os.replace(tmp, obj)
    return obj


def build(force: bool = False, verbose: bool = False) -> str:
    """Compile csrc/*.hip -> csrc/libgridenv.so for gfx950 (cross-compiles without a GPU):
    one object per source (cached by content hash), the sources compiled in parallel."""
    if not force and not needs_build():
        return LIB_PATH
    stamp = source_hash()  # of the sources as compiled (an edit during the build leaves it stale)
    if force and os.path.isdir(OBJ_DIR):
        for old in os.listdir(OBJ_DIR):
            os.remove(os.path.join(OBJ_DIR, old))
    from concurrent.futures import ThreadPoolExecutor
    with ThreadPoolExecutor(len(HIP_SOURCES)) as ex:
        objs = list(ex.map(lambda s: _object(s, verbose), HIP_SOURCES))
    tmp = LIB_PATH + f".tmp{os.getpid()}"
    cmd = [HIPCC, *HIPCC_FLAGS, *objs, "-o", tmp]
    if verbose:
        print(" ".join(cmd), flush=True)
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise GwError(f"hipcc link failed ({r.returncode}):\n{r.stderr[-4000:]}")
    os.replace(tmp, LIB_PATH)
    with open(STAMP_PATH, "w") as f:
        f.write(stamp)
    return LIB_PATH


class GwScenario(C.Structure):
    _fields_ = [("H", C.c_int32), ("W", C.c_int32), ("region", C.c_void_p),
                ("policy_id", C.c_void_p), ("n_policies", C.c_int32), ("policy_cdf", C.c_void_p),
                ("mdr", C.c_void_p), ("apples", C.c_void_p)]


class GwConfig(C.Structure):
    _fields_ = [("N", C.c_int32), ("K", C.c_int32), ("num_envs", C.c_int64),
                ("env_offset", C.c_int64), ("fear", C.c_int32), ("fear_weight", C.c_double),
                ("max_steps", C.c_int32), ("auto_reset", C.c_int32), ("seed", C.c_uint64),
                ("variant", C.c_int32)]


STEP_OUT_FIELDS = ["obs", "final_obs", "reward", "fear", "shaped", "term", "trunc", "done", "mask",
                   "crashes", "apples", "ep_return", "ep_fear", "ep_len", "actions", "mdr",
                   "final_pos", "crash_bits", "restr_bits", "stats", "done_copy", "stats_acc", "tick",
                   "desc_copy"]
GW_STATS = 8
STATS_NAMES = ["done_return", "episodes", "fear", "crashes", "apples", "shaped", "done_len", "env_steps"]


class GwStepOut(C.Structure):
    _fields_ = [(n, C.c_void_p) for n in STEP_OUT_FIELDS]


STATE_FIELDS = ["pos", "flags", "t", "episode", "prev_dist", "score", "fear_score"]


class GwState(C.Structure):
    _fields_ = [(n, C.c_void_p) for n in STATE_FIELDS]


EXPORTS = ["gw_create", "gw_reset", "gw_step", "gw_state_view", "gw_copy_state", "gw_profile",
           "gw_profile_read", "gw_stats_rows", "gw_dims", "gw_last_error", "gw_destroy", "gw_fear_matrix",
           "gw_adam_step", "gw_soft_update", "gw_obs_view", "gw_set_last_error", "gw_actor_act",
           "gw_actor_workspace_floats", "gw_actor_prepare", "gw_rollout_tick", "gw_set_obs_async",
           "gw_obs_fence", "gw_fear_fence", "gw_set_obs_dtype", "gw_set_fear_blocks", "gw_cnn_workspace_floats", "gw_cnn_prepare",
           "gw_cnn_act", "gw_return_compact", "gw_return_compact_scratch", "gw_kernel_path", "gw_graph_replayed", "gw_obs_patch", "gw_step_patch_next",
           "gw_ln_relu_fwd", "gw_ln_relu_bwd", "gw_gumbel_softmax",
           "gw_replay_gather", "gw_affine_relu_fwd", "gw_affine_relu_bwd",
           "gw_soft_update2", "gw_td_target", "gw_mean_loss_fwd", "gw_mean_loss_bwd",
           "gw_eval_accum", "gw_profile_spans", "gw_patch_actor_workspace_floats", "gw_patch_actor_prepare",
           "gw_patch_actor_act", "gw_patch_cnn_workspace_floats", "gw_patch_cnn_prepare", "gw_patch_cnn_act", "gw_patch_cnn_write_list", "gw_patch_cnn_act_listed",
           "gw_maddpg_workspace_floats", "gw_maddpg_critic_grads", "gw_maddpg_actor_grads",
           "gw_pipeline_state_bytes", "gw_pipeline_save", "gw_pipeline_load",
           "gw_gather_pack_scratch", "gw_gather_pack", "gw_gather_unpack_plan_cap", "gw_gather_unpack",
           "gw_adam_soft_step", "gw_obs_desc_copy", "gw_replay_gather_desc",
           "gw_maddpg_desc_workspace_floats", "gw_maddpg_desc_prime", "gw_maddpg_desc_update", "gw_count_sims",
           "gw_actor_images_view", "gw_maddpg_desc_update_img"]


class GwObsSource(C.Structure):
    _fields_ = [("desc", C.c_void_p), ("base", C.c_void_p), ("apples", C.c_int32 * GW_MAX_AGENTS),
                ("N", C.c_int32), ("K", C.c_int32), ("H", C.c_int32), ("W", C.c_int32), ("variant", C.c_int32),
                ("E", C.c_int64), ("env_offset", C.c_int64)]


MLP_PARAM_FIELDS = ["w1", "b1", "ln1_w", "ln1_b", "w2", "b2", "ln2_w", "ln2_b", "w3", "b3"]


class GwMlpActors(C.Structure):
    _fields_ = [("K", C.c_int32), ("in_dim", C.c_int32), ("hidden", C.c_int32), ("n_actions", C.c_int32),
                ("layer_norm", C.c_int32)] + [(n, C.c_void_p) for n in MLP_PARAM_FIELDS]


CNN_PARAM_FIELDS = ["conv1_w", "conv1_b", "conv2_w", "conv2_b", "lin1_w", "lin1_b", "w2", "b2", "w3", "b3"]


class GwCnnActors(C.Structure):
    _fields_ = [("K", C.c_int32), ("H", C.c_int32), ("W", C.c_int32), ("c1", C.c_int32), ("c2", C.c_int32),
                ("hidden", C.c_int32), ("n_actions", C.c_int32)] + [(n, C.c_void_p) for n in CNN_PARAM_FIELDS]


class GwMaddpgBatch(C.Structure):
    _fields_ = [("K", C.c_int32), ("B", C.c_int32), ("D", C.c_int32), ("x", C.c_void_p), ("x_next", C.c_void_p),
                ("reward", C.c_void_p), ("done", C.c_void_p), ("u", C.c_void_p), ("seed", C.c_uint64),
                ("ctr", C.c_void_p)]


class GwAdamBuf(C.Structure):
    _fields_ = [("param", C.c_void_p), ("grad", C.c_void_p), ("exp_avg", C.c_void_p), ("exp_avg_sq", C.c_void_p),
                ("step", C.c_void_p), ("n", C.c_int64), ("lr", C.c_double), ("beta1", C.c_double),
                ("beta2", C.c_double), ("eps", C.c_double)]


class GwActorImages(C.Structure):
    _fields_ = [("part", C.c_void_p), ("nslices", C.c_int32), ("w2img", C.c_void_p), ("w2bimg", C.c_void_p),
                ("w3img", C.c_void_p)]


class GwDescRing(C.Structure):
    _fields_ = [("desc", C.c_void_p), ("probs", C.c_void_p), ("reward", C.c_void_p), ("term", C.c_void_p),
                ("done", C.c_void_p), ("t_dev", C.c_void_p), ("S", C.c_int64)]


def _declare(L):
    p = C.c_void_p
    L.gw_maddpg_desc_workspace_floats.argtypes = [C.c_int32] * 4
    L.gw_maddpg_desc_workspace_floats.restype = C.c_int64
    L.gw_maddpg_desc_prime.argtypes = [C.POINTER(GwObsSource)] + [C.POINTER(GwMlpActors)] * 4 + [C.c_int32, p, p]
    L.gw_maddpg_desc_prime.restype = C.c_int
    L.gw_maddpg_desc_update.argtypes = [C.POINTER(GwObsSource), C.POINTER(GwDescRing)] + \
        [C.POINTER(GwMlpActors)] * 4 + [C.POINTER(GwAdamBuf)] * 2 + [p, p, C.c_float, C.c_float, C.c_int32,
                                                                     C.c_uint64, p, p, p, p, p]
    L.gw_maddpg_desc_update.restype = C.c_int
    L.gw_maddpg_desc_update_img.argtypes = [C.POINTER(GwObsSource), C.POINTER(GwDescRing)] + \
        [C.POINTER(GwMlpActors)] * 4 + [C.POINTER(GwAdamBuf)] * 2 + [p, p, C.c_float, C.c_float, C.c_int32,
                                                                     C.c_uint64, p, p, p, C.POINTER(GwActorImages), p, p]
    L.gw_maddpg_desc_update_img.restype = C.c_int
    L.gw_actor_images_view.argtypes = [p, C.c_int32, C.c_int32, C.POINTER(GwActorImages)]
    L.gw_actor_images_view.restype = C.c_int
    L.gw_maddpg_workspace_floats.argtypes = [C.c_int32, C.c_int32, C.c_int32]
    L.gw_maddpg_workspace_floats.restype = C.c_int64
    L.gw_maddpg_critic_grads.argtypes = [C.POINTER(GwMlpActors)] * 4 + [C.POINTER(GwMaddpgBatch), C.c_float, p, p, p, p]
    L.gw_maddpg_critic_grads.restype = C.c_int
    L.gw_maddpg_actor_grads.argtypes = [C.POINTER(GwMlpActors)] * 3 + [C.POINTER(GwMaddpgBatch), p, p, p, p, p]
    L.gw_maddpg_actor_grads.restype = C.c_int
    L.gw_cnn_workspace_floats.argtypes = [C.c_int32, C.c_int32, C.c_int32, C.c_int64]
    L.gw_cnn_workspace_floats.restype = C.c_int64
    L.gw_cnn_prepare.argtypes = [p, C.POINTER(GwCnnActors), p, p]
    L.gw_cnn_prepare.restype = C.c_int
    L.gw_cnn_act.argtypes = [p, C.POINTER(GwCnnActors), p, C.c_int, C.c_float, C.c_uint64, C.c_uint64,
                             p, p, p, p, p, p, p]
    L.gw_cnn_act.restype = C.c_int
    L.gw_create.argtypes = [C.POINTER(GwScenario), C.POINTER(GwConfig), C.c_int, C.POINTER(C.c_void_p)]
    L.gw_create.restype = C.c_int
    L.gw_reset.argtypes = [p, p, p, p, p, p]
    L.gw_reset.restype = C.c_int
    L.gw_step.argtypes = [p, p, p, p, C.POINTER(GwStepOut), p]
    L.gw_step.restype = C.c_int
    L.gw_state_view.argtypes = [p, C.POINTER(GwState)]
    L.gw_state_view.restype = C.c_int
    L.gw_copy_state.argtypes = [p, C.POINTER(GwState), C.c_int, p]
    L.gw_copy_state.restype = C.c_int
    L.gw_profile.argtypes = [p, C.c_int]
    L.gw_profile.restype = C.c_int
    L.gw_profile_read.argtypes = [p, C.POINTER(C.c_double), C.POINTER(C.c_int64)]
    L.gw_profile_read.restype = C.c_int
    L.gw_profile_spans.argtypes = [p, C.POINTER(C.c_double), C.c_int64, C.POINTER(C.c_int64)]
    L.gw_profile_spans.restype = C.c_int
    L.gw_obs_patch.argtypes = [p, C.c_int32, p, p, p]
    L.gw_obs_patch.restype = C.c_int
    L.gw_step_patch_next.argtypes = [p, C.c_int32, p, p]
    L.gw_step_patch_next.restype = C.c_int
    L.gw_gather_pack_scratch.argtypes = [C.c_int64]
    L.gw_gather_pack_scratch.restype = C.c_int64
    L.gw_gather_pack.argtypes = [p, p, C.c_int64, C.c_int64, p, C.c_int64, p, p, p, p]
    L.gw_gather_pack.restype = C.c_int
    L.gw_gather_unpack_plan_cap.argtypes = [C.c_int64, C.c_int32, C.c_int64]
    L.gw_gather_unpack_plan_cap.restype = C.c_int64
    L.gw_gather_unpack.argtypes = [p, C.c_int64, C.c_int32, C.c_int64, p, C.c_int64, p, p, C.c_int64, p,
                                   C.c_int64, p, C.c_int64, p, p]
    L.gw_gather_unpack.restype = C.c_int
    L.gw_pipeline_state_bytes.argtypes = []
    L.gw_pipeline_state_bytes.restype = C.c_int64
    L.gw_pipeline_save.argtypes = [p, p]
    L.gw_pipeline_save.restype = C.c_int
    L.gw_pipeline_load.argtypes = [p, p, p]
    L.gw_pipeline_load.restype = C.c_int
    L.gw_graph_replayed.argtypes = [p, p]
    L.gw_graph_replayed.restype = C.c_int
    L.gw_kernel_path.argtypes = [p]
    L.gw_kernel_path.restype = C.c_int64
    L.gw_stats_rows.argtypes = [p]
    L.gw_stats_rows.restype = C.c_int64
    L.gw_dims.argtypes = [p, C.POINTER(C.c_int64)]
    L.gw_dims.restype = C.c_int
    L.gw_last_error.argtypes = []
    L.gw_last_error.restype = C.c_char_p
    L.gw_fear_matrix.argtypes = [p, C.c_int64] + [p] * 11
    L.gw_fear_matrix.restype = C.c_int
    L.gw_adam_step.argtypes = [p, p, p, p, p, C.c_int64, C.c_double, C.c_double, C.c_double, C.c_double, C.c_int32, p]
    L.gw_adam_step.restype = C.c_int
    L.gw_adam_soft_step.argtypes = [p, p, p, p, p, C.c_int64, C.c_double, C.c_double, C.c_double, C.c_double, p,
                                    C.c_float, p, p, C.c_int64, C.c_int32, p]
    L.gw_adam_soft_step.restype = C.c_int
    L.gw_soft_update.argtypes = [p, p, C.c_int64, C.c_float, p]
    L.gw_soft_update.restype = C.c_int
    L.gw_ln_relu_fwd.argtypes = [p, p, p, p, p, p, C.c_int32, C.c_int64, C.c_int32, C.c_float, p]
    L.gw_ln_relu_fwd.restype = C.c_int
    L.gw_ln_relu_bwd.argtypes = [p] * 9 + [C.c_int32, C.c_int64, C.c_int32, p]
    L.gw_ln_relu_bwd.restype = C.c_int
    L.gw_gumbel_softmax.argtypes = [p, p, p, C.c_int64, C.c_int32, C.c_float, C.c_float, C.c_int64, C.c_int64, p]
    L.gw_gumbel_softmax.restype = C.c_int
    L.gw_soft_update2.argtypes = [p, p, C.c_int64, p, p, C.c_int64, C.c_float, p]
    L.gw_soft_update2.restype = C.c_int
    L.gw_td_target.argtypes = [p, p, p, C.c_float, p, C.c_int32, C.c_int64, p]
    L.gw_td_target.restype = C.c_int
    L.gw_mean_loss_fwd.argtypes = [p, p, p, C.c_int32, C.c_int64, C.c_int32, p]
    L.gw_mean_loss_fwd.restype = C.c_int
    L.gw_mean_loss_bwd.argtypes = [p, p, p, p, C.c_int32, C.c_int64, C.c_int32, p]
    L.gw_mean_loss_bwd.restype = C.c_int
    L.gw_eval_accum.argtypes = [p] * 7 + [C.c_int64, C.c_int32, p]
    L.gw_eval_accum.restype = C.c_int
    L.gw_affine_relu_fwd.argtypes = [p, p, p, p, C.c_int32, C.c_int64, C.c_int32, p]
    L.gw_affine_relu_fwd.restype = C.c_int
    L.gw_affine_relu_bwd.argtypes = [p] * 7 + [C.c_int32, C.c_int64, C.c_int32, p]
    L.gw_affine_relu_bwd.restype = C.c_int
    L.gw_replay_gather.argtypes = [p, p, C.c_int32] + [p] * 7 + [C.c_int64, C.c_int32, C.c_int64, C.c_int64,
                                                                  C.c_int64] + [p] * 8 + [C.c_uint64, p, p]
    L.gw_replay_gather.restype = C.c_int
    L.gw_replay_gather_desc.argtypes = [C.POINTER(GwObsSource)] + [p] * 8 + [C.c_int64, C.c_int64] + [p] * 8 + \
        [C.c_uint64, p, p]
    L.gw_replay_gather_desc.restype = C.c_int
    L.gw_count_sims.argtypes = [p, p]
    L.gw_count_sims.restype = C.c_int
    L.gw_obs_desc_copy.argtypes = [p, p, p]
    L.gw_obs_desc_copy.restype = C.c_int
    L.gw_obs_view.argtypes = [p, C.POINTER(GwObsSource)]
    L.gw_obs_view.restype = C.c_int
    L.gw_set_last_error.argtypes = [C.c_char_p]
    L.gw_set_last_error.restype = None
    L.gw_actor_act.argtypes = [p, C.POINTER(GwMlpActors), p, C.c_int, C.c_float, C.c_uint64, C.c_uint64,
                               p, p, p, p, p, p, p]
    L.gw_actor_act.restype = C.c_int
    L.gw_patch_actor_workspace_floats.argtypes = [C.c_int32, C.c_int32, C.c_int32, C.c_int32]
    L.gw_patch_actor_workspace_floats.restype = C.c_int64
    L.gw_patch_actor_prepare.argtypes = [p, C.c_int32, C.POINTER(GwMlpActors), p, p]
    L.gw_patch_actor_prepare.restype = C.c_int
    L.gw_patch_actor_act.argtypes = [p, C.c_int32, C.POINTER(GwMlpActors), p, C.c_int, C.c_float, C.c_uint64,
                                     C.c_uint64, p, p, p, p, p, p, p]
    L.gw_patch_actor_act.restype = C.c_int
    L.gw_patch_cnn_workspace_floats.argtypes = [C.c_int32, C.c_int32, C.c_int32, C.c_int32, C.c_int64]
    L.gw_patch_cnn_workspace_floats.restype = C.c_int64
    L.gw_patch_cnn_prepare.argtypes = [p, C.c_int32, C.POINTER(GwCnnActors), p, p]
    L.gw_patch_cnn_prepare.restype = C.c_int
    L.gw_patch_cnn_act.argtypes = [p, C.c_int32, C.POINTER(GwCnnActors), p, C.c_int, C.c_float, C.c_uint64,
                                   C.c_uint64, p, p, p, p, p, p, p]
    L.gw_patch_cnn_act.restype = C.c_int
    L.gw_patch_cnn_act_listed.argtypes = L.gw_patch_cnn_act.argtypes
    L.gw_patch_cnn_act_listed.restype = C.c_int
    L.gw_patch_cnn_write_list.argtypes = [p, C.c_int32, C.POINTER(GwCnnActors), p, p, p, p]
    L.gw_patch_cnn_write_list.restype = C.c_int
    L.gw_actor_workspace_floats.argtypes = [C.c_int32, C.c_int32]
    L.gw_actor_workspace_floats.restype = C.c_int64
    L.gw_actor_prepare.argtypes = [p, C.POINTER(GwMlpActors), p, p]
    L.gw_actor_prepare.restype = C.c_int
    L.gw_rollout_tick.argtypes = [p, C.c_int64, C.c_int32, p, p, p, p]
    L.gw_rollout_tick.restype = C.c_int
    L.gw_return_compact.argtypes = [p, C.c_int64, C.c_int32, C.c_int64, C.c_int64, p, C.c_int64, p, p, p]
    L.gw_return_compact.restype = C.c_int
    L.gw_return_compact_scratch.argtypes = [C.c_int64, C.c_int32, C.c_int64]
    L.gw_return_compact_scratch.restype = C.c_int64
    L.gw_set_obs_async.argtypes = [p, C.c_int]
    L.gw_set_obs_async.restype = C.c_int
    L.gw_obs_fence.argtypes = [p, p]
    L.gw_obs_fence.restype = C.c_int
    L.gw_fear_fence.argtypes = [p, p]
    L.gw_fear_fence.restype = C.c_int
    L.gw_set_obs_dtype.argtypes = [p, C.c_int]
    L.gw_set_obs_dtype.restype = C.c_int
    L.gw_set_fear_blocks.argtypes = [p, C.c_int]
    L.gw_set_fear_blocks.restype = C.c_int
    L.gw_destroy.argtypes = [p]
    L.gw_destroy.restype = None
    return L


def load(build_if_needed: bool = True):
    """Load libgridenv.so (building it first if stale).  Imports torch first on purpose."""
    global _lib
    with _lock:
        if _lib is not None:
            return _lib
        import torch  # noqa: F401  (bind to torch's HIP runtime)
        alt = os.environ.get("MARLNAV_LIB")  # measurement builds only (tools/step_clk.sh)
        if alt:
            _lib = _declare(C.CDLL(alt))
            return _lib
        if build_if_needed and needs_build():
            build()
        if not os.path.exists(LIB_PATH):
            raise GwError(f"{LIB_PATH} is missing; run __graft_entry__.build()")
        _lib = _declare(C.CDLL(LIB_PATH))
        return _lib


def check(status: int, what: str):
    if status != 0:
        msg = load().gw_last_error().decode(errors="replace")
        raise GwError(f"{what} failed (status {status}): {msg}")


class RecordingError(RuntimeError):
    """A torch GPU kernel was launched inside a LaunchRecorder (it would be missing from replays)."""


def _no_torch_kernels_mode():
    import torch
    from torch.utils._python_dispatch import TorchDispatchMode

    # ops that launch no kernel: allocations and metadata queries (views are recognised by
    # OpOverload.is_view)
    free = {"empty", "empty_strided", "empty_like", "new_empty", "new_empty_strided", "detach", "lift_fresh",
            "sym_size", "sym_stride", "sym_numel", "sym_storage_offset", "is_same_size", "alias"}

    class Mode(TorchDispatchMode):
        def __torch_dispatch__(self, func, types, args=(), kwargs=None):
            kwargs = kwargs or {}
            name = func.overloadpacket.__name__
            if not (getattr(func, "is_view", False) or name in free):
                leaves = list(args) + list(kwargs.values())
                flat = []
                for a in leaves:
                    flat.extend(a if isinstance(a, (list, tuple)) else (a,))
                dev = kwargs.get("device")
                on_gpu = any(isinstance(a, torch.Tensor) and a.is_cuda for a in flat) or \
                    (dev is not None and torch.device(dev).type == "cuda")
                if on_gpu:
                    raise RecordingError(f"LaunchRecorder: torch op {func} would launch a GPU kernel that "
                                         "replays of the recording would miss")
            return func(*args, **kwargs)
    return Mode()


class LaunchRecorder:
    """Records the stream-ordered C-ABI calls made while active: every exported function whose
    last argument is ``stream`` (the handle of the stream being recorded).  ``replay(s)`` issues
    them again, in order, on stream ``s``, with the same arguments (ctypes structs passed by
    reference stay alive in the recorded tuples).  Used by MADDPG.capture(launches=True): the
    update runs once eagerly while recorded (its buffers come from the ordinary allocator; the
    caller keeps them alive for as long as it replays), then is re-issued as plain launches
    instead of a graph replay.

    A torch operation that would launch a kernel on the GPU while recording cannot be replayed
    (only C-ABI calls are recorded), so it raises ``RecordingError`` instead of being dropped
    silently (``forbid_torch``, the default): views, allocations and host-side work are allowed."""

    def __init__(self, stream: int, forbid_torch: bool = True):
        self.stream = int(stream)
        self.calls = []
        self._saved = {}
        self._mode = _no_torch_kernels_mode() if forbid_torch else None

    def __enter__(self):
        if self._mode is not None:
            self._mode.__enter__()
        L = load()
        for name in EXPORTS:
            f = getattr(L, name, None)
            if f is None or name in self._saved:
                continue
            self._saved[name] = f
            setattr(L, name, self._wrap(name, f))
        return self

    def __exit__(self, *exc):
        L = load()
        for name, f in self._saved.items():
            setattr(L, name, f)
        self._saved = {}
        if self._mode is not None:
            self._mode.__exit__(*exc)
        return False

    def _wrap(self, name, f):
        def call(*args):
            last = args[-1] if args else None
            if isinstance(last, C.c_void_p):
                last = last.value
            if isinstance(last, int) and last == self.stream:
                self.calls.append((name, f, args[:-1]))
            return f(*args)
        return call

    def replay(self, stream: int):
        for name, f, args in self.calls:
            status = f(*args, stream)
            if status:
                check(status, name)
