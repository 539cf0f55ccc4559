"""ctypes binding of libg2048.so (include/g2048.h) -- the only way this package reaches the GPU.

There is no fallback: if the library is missing, or no HIP device is present, every entry point raises.
torch is imported before the library is opened so that the library's libamdhip64 dependency resolves to the
HIP runtime torch already loaded (same SONAME), i.e. one HIP context shared with torch's allocator/streams.
"""
from __future__ import annotations

import ctypes
import os
import subprocess
import threading

import torch

PKG_DIR = os.path.dirname(os.path.abspath(__file__))
REPO_ROOT = os.path.dirname(PKG_DIR)
SHIPPED_LIB = os.path.join(PKG_DIR, "libg2048.so")
LIB_PATH = SHIPPED_LIB
SRC = os.path.join(PKG_DIR, "csrc", "g2048.hip")
SOURCES = [SRC, os.path.join(PKG_DIR, "csrc", "g2048_policy.hip"), os.path.join(PKG_DIR, "csrc", "g2048_dw2.hip"),
           os.path.join(PKG_DIR, "csrc", "g2048_deep.hip")]
INCLUDE = os.path.join(REPO_ROOT, "include")
ABI_VERSION = 16
DEEP_MAX_HIDDEN = 4

# include/g2048.h constants
OBS_NONE, OBS_RAW, OBS_LOG2, OBS_ONEHOT = -1, 0, 1, 2
ACT_RELU, ACT_SIGMOID = 0, 1
RNG_PCG64, RNG_PHILOX = 0, 1
F_CHANGED, F_TERMINATED, F_TRUNCATED, F_INVALID = 0x01, 0x02, 0x04, 0x08
F_OVERFLOW, F_RESET, F_INACTIVE, F_BADACTION = 0x10, 0x20, 0x40, 0x80
# lane state word (g2048_lanes.state)
LS_STEP_MASK, LS_MAXT_SHIFT, LS_ACTIVE, LS_HAS_U32 = 0x000FFFFF, 20, 0x02000000, 0x04000000
MAX_STEPS_LIMIT = 0x000FFFFF
G2048_OK, G2048_EINVAL, G2048_EHIP, G2048_ENOINIT = 0, 1, 2, 3


CSRC = os.path.join(PKG_DIR, "csrc")
BUILD_DIR = os.path.join(PKG_DIR, "build")
# -ffp-contract=off: the fp64 reward keeps the reference's separately rounded multiply and add (no FMA)
HIPCC_FLAGS = ["--offload-arch=gfx950", "-O3", "-std=c++17", "-ffp-contract=off", "-fPIC"]


_COMPILER_ID: str | None = None


def _compiler_id() -> str:
    """The resolved hipcc and its version text: part of every object's cache key, so a ROCm / hipcc change
    rebuilds instead of linking objects from another compiler."""
    global _COMPILER_ID
    if _COMPILER_ID is None:
        import shutil

        exe = shutil.which("hipcc") or "hipcc"
        r = subprocess.run([exe, "--version"], capture_output=True, text=True)
        _COMPILER_ID = os.path.realpath(exe) + "\n" + r.stdout + r.stderr
    return _COMPILER_ID


def _object_for(src: str, flags: list[str]) -> str:
    """build/<tu>-<hash>.o: keyed by the TU, every header it may include, the flags and the compiler
    (incremental builds)."""
    import hashlib

    h = hashlib.sha256(" ".join(flags).encode())
    h.update(_compiler_id().encode())
    hdrs = sorted(os.path.join(CSRC, f) for f in os.listdir(CSRC) if f.endswith((".h", ".inc")))
    for f in [src] + hdrs + [os.path.join(INCLUDE, "g2048.h")]:
        with open(f, "rb") as fh:
            h.update(fh.read())
    return os.path.join(BUILD_DIR, f"{os.path.splitext(os.path.basename(src))[0]}-{h.hexdigest()[:16]}.o")


def build(verbose: bool = False, out: str | None = None, defines: tuple[str, ...] = (),
          define_tus: tuple[str, ...] | None = None) -> str:
    """Compile libg2048.so for gfx950 in-tree (hipcc cross-compiles; no GPU needed).  Every TU is compiled to an
    object in parallel (cached under build/ by content hash), then linked.  out / defines (applied to the TUs
    named in define_tus, default all): tools-only variant builds (e.g. the -DG2048_DIAG=1 timing build); the
    product is the default."""
    from concurrent.futures import ThreadPoolExecutor

    os.makedirs(BUILD_DIR, exist_ok=True)
    base_flags = HIPCC_FLAGS + ["-I" + INCLUDE, "-I" + CSRC]

    def compile_one(src):
        use_defs = define_tus is None or os.path.basename(src) in define_tus
        flags = base_flags + ([f"-D{d}" for d in defines] if use_defs else [])
        obj = _object_for(src, flags)
        if not os.path.exists(obj):
            tmp = obj + f".tmp{os.getpid()}"
            cmd = ["hipcc"] + flags + ["-c", src, "-o", tmp]
            r = subprocess.run(cmd, capture_output=True, text=True)
            if r.returncode != 0:
                raise RuntimeError("hipcc failed:\n" + " ".join(cmd) + "\n" + r.stdout + r.stderr)
            os.replace(tmp, obj)
        return obj

    with ThreadPoolExecutor(max_workers=min(8, len(SOURCES))) as ex:
        objs = list(ex.map(compile_one, SOURCES))
    target = out or SHIPPED_LIB
    cmd = ["hipcc", "--offload-arch=gfx950", "-shared", "-fPIC", "-o", target] + objs
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError("link failed:\n" + r.stdout + r.stderr)
    if verbose:
        print(" ".join(cmd))
    return target


class EnvCfg(ctypes.Structure):
    _fields_ = [("obs_mode", ctypes.c_int32), ("reward_mode", ctypes.c_int32), ("bonus_mode", ctypes.c_int32),
                ("use_action_mask", ctypes.c_int32), ("obs_log2_scale", ctypes.c_float), ("_pad0", ctypes.c_int32),
                ("base_reward_scale", ctypes.c_double), ("empty_tile_reward", ctypes.c_double),
                ("merge_reward", ctypes.c_double), ("bonus_scale", ctypes.c_double), ("step_reward", ctypes.c_double),
                ("endgame_penalty", ctypes.c_double), ("invalid_action_penalty", ctypes.c_double),
                ("max_steps", ctypes.c_int64)]


class Lanes(ctypes.Structure):
    _fields_ = [(name, ctypes.c_void_p) for name in
                ("board", "state", "seed", "rng_state", "rng_inc", "rng_uint")]


class StepOut(ctypes.Structure):
    _fields_ = [(name, ctypes.c_void_p) for name in ("reward", "flags", "mask", "obs", "merged", "prev_board",
                                                         "reward64", "score_add", "mask_bits")]


class Traj(ctypes.Structure):
    _fields_ = [(name, ctypes.c_void_p) for name in ("boards", "actions", "rewards", "flags", "probs", "lengths",
                                                     "totals", "max_tile", "final_board")]


class TdRows(ctypes.Structure):
    """g2048_td_rows: the per-row critic pass's TD target inputs (lane-indexed V(s') in, V(s) out)."""
    _fields_ = [("lane", ctypes.c_void_p), ("reward", ctypes.c_void_p), ("has_next", ctypes.c_void_p),
                ("v_next", ctypes.c_void_p), ("v_out", ctypes.c_void_p), ("gamma", ctypes.c_float),
                ("reserved", ctypes.c_int32)]


class Suspend(ctypes.Structure):
    _fields_ = [(name, ctypes.c_void_p) for name in ("board", "meta", "total", "list", "count")]


_lib = None
_lock = threading.RLock()
_inited_devices: set[int] = set()


def _declare(L):
    vp, i64, u64, i32, d, f = ctypes.c_void_p, ctypes.c_int64, ctypes.c_uint64, ctypes.c_int, ctypes.c_double, ctypes.c_float
    P = ctypes.POINTER
    L.g2048_abi_version.restype = ctypes.c_int
    L.g2048_last_error.restype = ctypes.c_char_p
    L.g2048_init.argtypes = [i32]
    L.g2048_seed_pcg64.argtypes = [vp, vp, vp, vp, i64, vp]
    L.g2048_reset.argtypes = [P(Lanes), vp, vp, P(EnvCfg), i32, u64, vp, vp, i64, vp]
    L.g2048_step.argtypes = [P(Lanes), vp, P(EnvCfg), P(StepOut), i32, u64, i32, u64, i64, vp]
    L.g2048_obs.argtypes = [vp, i32, f, vp, vp, i64, vp]
    L.g2048_move.argtypes = [vp, vp, vp, vp, vp, i64, vp]
    L.g2048_sample.argtypes = [vp, vp, vp, i32, i32, vp, vp, vp, u64, vp, vp, vp, i64, vp]
    L.g2048_returns.argtypes = [vp, vp, d, vp, i64, i64, vp]
    L.g2048_symmetries.argtypes = [vp, vp, vp, vp, i64, vp]
    L.g2048_policy_packed_size.argtypes = [i32, i32]
    L.g2048_policy_packed_size.restype = i64
    L.g2048_policy_pack.argtypes = [vp, vp, vp, vp, vp, vp, i32, i32, i32, vp, i64, vp]
    L.g2048_policy.argtypes = [vp, i32, i32, i32, vp, vp, vp, i32, f, i32, i32, i32, vp, vp, vp, u64, vp, vp, vp, vp,
                               i64, vp]
    L.g2048_rollout.argtypes = [vp, i32, i32, i32, P(EnvCfg), i32, vp, vp, vp, vp, vp, vp, vp, i64, i64, vp, vp, vp, vp,
                                vp, vp, vp, vp, vp, vp]
    L.g2048_grad_packed_size.argtypes = [i32, i32]
    L.g2048_grad_packed_size.restype = i64
    L.g2048_grad_partial_size.argtypes = [i32, i32]
    L.g2048_grad_partial_size.restype = i64
    L.g2048_grad_pack.argtypes = [vp, i32, i32, vp, i64, vp]
    L.g2048_actor_grad_waves.argtypes = []
    L.g2048_actor_grad.argtypes = [vp, vp, i32, i32, i32, i32, f, i32, vp, vp, vp, i64, i64, vp, vp, vp, i64, i32, vp]
    L.g2048_critic_grad.argtypes = [vp, vp, i32, i32, i32, i32, f, i32, f, vp, vp, vp, vp, vp, i64, i64, i64, i64, vp, vp,
                                    vp, i32, i64, i32, P(TdRows), vp]
    L.g2048_dw2.argtypes = [vp, vp, i32, i32, i64, i64, i64, i64, vp, i64, vp]
    L.g2048_fold_partials.argtypes = [vp, i64, i64, vp, vp]
    L.g2048_dw2_factored.argtypes = [vp, vp, vp, i32, i32, i64, i64, i64, i64, vp, i64, vp]
    L.g2048_dw2_actor.argtypes = [vp, vp, vp, i32, i32, i64, i64, i64, i64, vp, i64, vp]
    L.g2048_deep_packed_size.argtypes = [i32, i32, vp]
    L.g2048_deep_packed_size.restype = i64
    L.g2048_deep_pack.argtypes = [vp, vp, i32, i32, vp, i32, vp, i64, vp]
    L.g2048_deep_policy.argtypes = [vp, i32, vp, i32, vp, vp, vp, i32, f, i32, i32, i32, vp, vp, vp, u64, vp, vp, vp,
                                    vp, i64, vp]
    L.g2048_deep_rollout.argtypes = [vp, i32, vp, i32, P(EnvCfg), i32, vp, vp, vp, vp, vp, vp, vp, vp, i64, i32,
                                     P(Suspend), i64, i64, P(Traj), vp]
    L.g2048_deep_hidden.argtypes = [vp, i32, vp, i32, i32, f, vp, i64, i32, vp, i64, vp]
    L.g2048_deep_grad_pack_size.argtypes = [i32, i32, vp]
    L.g2048_deep_grad_pack_size.restype = i64
    L.g2048_deep_grad_slab.argtypes = [i32, i32, vp]
    L.g2048_deep_grad_slab.restype = i64
    L.g2048_deep_grad_parts.argtypes = [i32, i32, vp]
    L.g2048_deep_grad_parts.restype = i32
    L.g2048_deep_grad_passes.argtypes = [i32, i32, vp]
    L.g2048_deep_grad_passes.restype = i32
    L.g2048_deep_grad_pack.argtypes = [vp, i32, i32, vp, vp, i64, vp]
    L.g2048_deep_grad.argtypes = [vp, vp, i32, vp, i32, i32, f, i32, vp, vp, vp, i32, i32, f, vp, vp, vp, vp, i64, vp,
                                  i64, P(TdRows), vp]
    L.g2048_onehot_layer1.argtypes = [vp, vp, i32, i32, vp, i64, i64, vp, vp]
    L.g2048_onehot_dw1_slab.argtypes = [i32]
    L.g2048_onehot_dw1_slab.restype = i64
    L.g2048_onehot_dw1.argtypes = [vp, vp, i32, i64, i64, i64, vp, i64, vp]
    for name in ("g2048_init", "g2048_seed_pcg64", "g2048_reset", "g2048_step", "g2048_obs", "g2048_move",
                 "g2048_sample", "g2048_returns", "g2048_symmetries", "g2048_policy_pack", "g2048_policy",
                 "g2048_rollout", "g2048_grad_pack", "g2048_actor_grad_waves", "g2048_actor_grad", "g2048_critic_grad",
                 "g2048_dw2", "g2048_fold_partials", "g2048_dw2_factored", "g2048_dw2_actor", "g2048_deep_pack", "g2048_deep_policy",
                 "g2048_deep_rollout", "g2048_deep_hidden", "g2048_deep_grad_pack", "g2048_deep_grad",
                 "g2048_onehot_layer1", "g2048_onehot_dw1"):
        getattr(L, name).restype = ctypes.c_int


EXPORTED_SYMBOLS = ("g2048_abi_version", "g2048_last_error", "g2048_init", "g2048_seed_pcg64", "g2048_reset",
                    "g2048_step", "g2048_obs", "g2048_move", "g2048_sample", "g2048_returns", "g2048_symmetries",
                    "g2048_policy_packed_size", "g2048_policy_pack", "g2048_policy", "g2048_rollout",
                    "g2048_grad_packed_size", "g2048_grad_partial_size", "g2048_grad_pack", "g2048_actor_grad_waves",
                    "g2048_actor_grad", "g2048_critic_grad", "g2048_dw2", "g2048_fold_partials",
                    "g2048_dw2_factored", "g2048_dw2_actor", "g2048_deep_packed_size", "g2048_deep_pack", "g2048_deep_policy",
                    "g2048_deep_rollout", "g2048_deep_hidden", "g2048_deep_grad_pack_size", "g2048_deep_grad_slab",
                    "g2048_deep_grad_parts", "g2048_deep_grad_passes",
                    "g2048_deep_grad_pack", "g2048_deep_grad", "g2048_onehot_layer1", "g2048_onehot_dw1_slab",
                    "g2048_onehot_dw1")


def lib():
    """Open libg2048.so (no device work).  Raises if it is not built."""
    global _lib
    if _lib is not None:
        return _lib
    with _lock:
        if _lib is None:
            if not os.path.exists(LIB_PATH):
                raise RuntimeError(f"{LIB_PATH} is not built: run `python -c 'import __graft_entry__ as g; g.build()'`")
            L = ctypes.CDLL(LIB_PATH)
            _declare(L)
            v = L.g2048_abi_version()
            if v != ABI_VERSION:
                raise RuntimeError(f"libg2048.so ABI {v} != expected {ABI_VERSION}; rebuild")
            _lib = L
    return _lib


def use_library_for_tools(path: str) -> None:
    """tools/ only: open another build of the same ABI (the -DG2048_DIAG=1 timing-attribution build of
    tools/diag_build.sh) instead of the shipped library.  Must run before the first lib() call; the product
    path never calls it (nothing in the package reads the environment to switch libraries)."""
    global LIB_PATH
    if _lib is not None:
        raise RuntimeError("libg2048 is already open")
    LIB_PATH = os.path.abspath(path)


def check(rc: int) -> None:
    if rc == G2048_OK:
        return
    msg = lib().g2048_last_error().decode(errors="replace")
    if rc == G2048_EINVAL:
        raise ValueError(msg)
    raise RuntimeError(f"libg2048 error {rc}: {msg}")


def ensure_device(device: torch.device) -> None:
    """g2048_init for `device` (builds the row table there).  Fails loudly without a HIP device."""
    if device.type != "cuda":
        raise RuntimeError(f"the 2048 hot path runs on a HIP device only (got {device}); there is no CPU fallback")
    if not torch.cuda.is_available():
        raise RuntimeError("no HIP device visible: the 2048 hot path has no CPU fallback")
    idx = device.index if device.index is not None else torch.cuda.current_device()
    if idx in _inited_devices:
        return
    with _lock:
        if idx not in _inited_devices:
            check(lib().g2048_init(idx))
            _inited_devices.add(idx)


def stream_handle(device: torch.device) -> int:
    return torch.cuda.current_stream(device).cuda_stream


def ptr(t: torch.Tensor | None) -> int | None:
    if t is None:
        return None
    if not t.is_contiguous():
        raise ValueError("buffers passed to libg2048 must be contiguous")
    return t.data_ptr()
