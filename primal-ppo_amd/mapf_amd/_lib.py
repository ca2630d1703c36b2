"""ctypes binding of libmapf.so (include/mapf.h).

This is the binding a maintainer of the reference would add;
every entry point declared in include/mapf.h is bound here with its exact
C signature.  Loading fails loudly when the library is missing.
"""
import ctypes
import os

from .config import MapfConfig

PKG = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB_PATH = os.environ.get("MAPF_LIB", os.path.join(PKG, "lib", "libmapf.so"))

P = ctypes.c_void_p
I32 = ctypes.c_int32
U32 = ctypes.c_uint32
I64 = ctypes.c_int64
F32 = ctypes.c_float


class ResetSpec(ctypes.Structure):
    _fields_ = [("mode", I32), ("reserved", I32), ("maps", P), ("seq", P), ("seq_len", P),
                ("human_start", P), ("human_goal", P), ("human_seq", P), ("human_seq_len", P),
                ("seed", ctypes.c_uint64)]


class MapGenSpec(ctypes.Structure):
    """include/mapf.h: mapf_mapgen_spec."""
    _fields_ = [("kind", I32), ("lo", I32), ("hi", I32), ("largest", I32), ("density", ctypes.c_float),
                ("epoch", U32), ("seed", ctypes.c_uint64)]


MAPS_WAREHOUSE, MAPS_RANDOM = 0, 1


class StepOut(ctypes.Structure):
    _fields_ = [(n, P) for n in ("status", "reward", "shadow_goals", "cost", "train_valid", "actions_fixed",
                                 "goals_reached", "constraints", "reward_total")]


class State(ctypes.Structure):
    _fields_ = [(n, P) for n in ("pos", "goal", "last_action", "seq_cursor", "human", "human_path", "clock")]


TUNING_FIELDS = ("roll_occ", "roll_group", "roll_fair", "roll_slack", "wide_nt", "wide_pipe", "wide_grid",
                 "wide_overlap", "wide_obs", "wide_epw", "wide_pair", "wide_slack", "wide_fair", "wide_prio",
                 "wide_bfsobs", "xcd_remap", "obs_envs", "step_block", "search_blocks", "band_blocks", "agent_lanes",
                 "serial_search", "no_defer", "diag_exp")


class Tuning(ctypes.Structure):
    """include/mapf.h: mapf_tuning (launch forms; identical results whatever the values)."""
    _fields_ = [(n, I32) for n in TUNING_FIELDS]


# name -> (restype, argtypes)
SIGNATURES = {
    "mapf_last_error": (ctypes.c_char_p, []),
    "mapf_abi_version": (ctypes.c_int, []),
    "mapf_create": (ctypes.c_int, [ctypes.POINTER(MapfConfig), ctypes.c_int, ctypes.POINTER(P)]),
    "mapf_destroy": (ctypes.c_int, [P]),
    "mapf_path_capacity": (ctypes.c_int, [P]),
    "mapf_step_observe_fused": (ctypes.c_int, [P]),
    "mapf_reset": (ctypes.c_int, [P, ctypes.POINTER(ResetSpec), P]),
    "mapf_reset_generated": (ctypes.c_int, [P, ctypes.POINTER(MapGenSpec), P, P]),
    "mapf_step": (ctypes.c_int, [P, P, ctypes.POINTER(StepOut), U32, P]),
    "mapf_step_random": (ctypes.c_int, [P, P, ctypes.POINTER(StepOut), U32, P]),
    "mapf_observe": (ctypes.c_int, [P, P, P, P]),
    "mapf_step_observe": (ctypes.c_int, [P, P, ctypes.POINTER(StepOut), P, P, P]),
    "mapf_step_observe_random": (ctypes.c_int, [P, P, ctypes.POINTER(StepOut), P, P, P]),
    "mapf_rollout_random": (ctypes.c_int, [P, I32, I32, P, ctypes.POINTER(StepOut), P, P, P]),
    "mapf_rollout_random_fused": (ctypes.c_int, [P]),
    "mapf_tuning_default": (None, [ctypes.POINTER(Tuning)]),
    "mapf_get_tuning": (ctypes.c_int, [P, ctypes.POINTER(Tuning)]),
    "mapf_set_tuning": (ctypes.c_int, [P, ctypes.POINTER(Tuning)]),
    "mapf_rollout_plan": (ctypes.c_int, [P, I32, ctypes.c_char_p, I32]),
    "mapf_flush": (ctypes.c_int, [P, P]),
    "mapf_release_captures": (ctypes.c_int, [P]),
    "mapf_random_actions": (ctypes.c_int, [P, P, P]),
    "mapf_bfs": (ctypes.c_int, [P, P, P]),
    "mapf_render": (ctypes.c_int, [P, P, I32, I32, P, P]),
    "mapf_get_counters": (ctypes.c_int, [P, P, P]),
    "mapf_get_profile": (ctypes.c_int, [P, P, ctypes.c_int, P]),
    "mapf_get_timeline": (ctypes.c_int, [P, P, ctypes.c_int32, P]),
    "mapf_get_wave_profile": (ctypes.c_int, [P, P, ctypes.c_int32, P]),
    "mapf_get_state": (ctypes.c_int, [P, ctypes.POINTER(State), P]),
    "mapf_set_state": (ctypes.c_int, [P, ctypes.POINTER(State), P]),
    "mapf_gae": (ctypes.c_int, [P, P, P, P, P, I32, I32, ctypes.c_double, ctypes.c_double, P]),
    "mapf_normalize_advantages": (ctypes.c_int, [P, P, P, P, P, P, I32, ctypes.c_double, I32, P]),
    "mapf_sample_actions": (ctypes.c_int, [P, I32, P, P, I32, ctypes.c_uint64, U32, P]),
    "mapf_advantage_moments": (ctypes.c_int, [P, P, P, P, I32, P, P, P]),
    "mapf_normalize_advantages_stats": (ctypes.c_int, [P, P, P, P, P, P, P, I32, ctypes.c_double, I32, P]),
    "mapf_normalize_advantages_stats_dlam": (ctypes.c_int, [P, P, P, P, P, P, P, I32, P, I32, P]),
    "mapf_episode_sum": (ctypes.c_int, [P, I32, I32, I32, P, P]),
    # policy acting forward epilogues (csrc/mapf_policy.hip)
    "mapf_nhwc_bias_relu": (ctypes.c_int, [P, P, I64, I32, P]),
    "mapf_nhwc_bias_relu_pool2": (ctypes.c_int, [P, P, P, I32, I32, I32, I32, P]),
    "mapf_layernorm_f16": (ctypes.c_int, [P, I64, P, P, P, I64, I32, ctypes.c_float, P]),
    "mapf_colsum_f16": (ctypes.c_int, [P, P, P, I64, I32, P]),
    "mapf_relu_bias_pool_bwd_f16": (ctypes.c_int, [P, P, P, P, P, P, I32, I32, I32, I32, P]),
    "mapf_relu_bias_bwd_f16": (ctypes.c_int, [P, P, P, P, P, I64, I32, P]),
    "mapf_cast_f32_to_f16_multi": (ctypes.c_int, [P, P, P, I32, P]),
    "mapf_cast_f32_to_f16_multi_flip": (ctypes.c_int, [P, P, P, P, P, I32, P]),
    "mapf_tokens_layernorm_train": (ctypes.c_int, [P, P, P, P, P, I64, I32, F32, P, U32, P, P, F32, P, P]),
    "mapf_tokens_train_bwd": (ctypes.c_int, [P, P, P, P, P, P, P, P, I64, I32, F32, P, U32, P]),
    "mapf_optim_unscale_clip_adam": (ctypes.c_int, [P, P, P, P, P, P, I32, P, F32, F32, F32, F32, F32, P, P, P,
                                                    I64, P]),
    "mapf_cast_f16_to_f32_multi": (ctypes.c_int, [P, P, P, I32, P]),
    "mapf_layernorm_bwd_f16": (ctypes.c_int, [P, I64, P, P, P, P, P, P, P, I64, I32, ctypes.c_float, P]),
    "mapf_layernorm_dropout_bwd_f16": (ctypes.c_int, [P, P, P, P, P, P, P, P, P, I64, I32, F32, F32, P, U32, P]),
    "mapf_dropout_residual_layernorm_train": (ctypes.c_int, [P, I64, P, P, P, P, P, I64, I32, F32, F32, P, U32, P]),
    "mapf_gelu_dropout_train_f16": (ctypes.c_int, [P, P, I64, F32, P, U32, P]),
    "mapf_gelu_dropout_bwd_f16": (ctypes.c_int, [P, P, P, I64, F32, P, U32, P]),
    "mapf_dropout_residual": (ctypes.c_int, [P, P, I64, ctypes.c_float, ctypes.c_uint64, P]),
    "mapf_dropout_residual_layernorm": (ctypes.c_int, [P, P, P, P, P, I64, I32, ctypes.c_float, ctypes.c_float,
                                                        ctypes.c_uint64, P]),
    "mapf_gelu_dropout_f16": (ctypes.c_int, [P, I64, ctypes.c_float, ctypes.c_uint64, P]),
    "mapf_tokens": (ctypes.c_int, [P, P, P, P, P, I64, I32, I32, ctypes.c_float, ctypes.c_uint64, P]),
    "mapf_tokens_layernorm": (ctypes.c_int, [P, P, P, P, P, I64, I32, I32, ctypes.c_float, ctypes.c_uint64, P, P,
                                              ctypes.c_float, P, P]),
    "mapf_ppo_loss": (ctypes.c_int, [P, P, P, P, P, P, P, P, P, P, P, P, I32, P, I64, I32, P, P, P, P, P, P, P,
                                     P]),
    "mapf_ppo_loss_dcoef": (ctypes.c_int, [P, P, P, P, P, P, P, P, P, P, P, P, I32, P, I64, I32, P, P, P, P, P, P, P,
                                           P]),
    "mapf_normalize_advantages_dlam": (ctypes.c_int, [P, P, P, P, P, P, I32, P, I32, P]),
    "mapf_linear512_gelu_dropout": (ctypes.c_int, [P, P, P, P, I64, ctypes.c_float, ctypes.c_uint64, P]),
    "mapf_linear512_select": (ctypes.c_int, [I32]),
    "mapf_linear512_stages": (ctypes.c_int, [I32]),
    "mapf_linear512_kdepth": (ctypes.c_int, [I32]),
    "mapf_linear512_residual_layernorm": (ctypes.c_int, [P, P, P, P, P, P, P, I64, ctypes.c_float, ctypes.c_float,
                                                          ctypes.c_uint64, P]),
    "mapf_linear512_residual_layernorm_rows": (ctypes.c_int, [P, P, P, P, P, P, P, I64, ctypes.c_float,
                                                              ctypes.c_float, ctypes.c_uint64, I32, P]),
    "mapf_linear512_tokens_residual_layernorm": (ctypes.c_int, [P, P, P, P, P, P, P, I64, I32, ctypes.c_float,
                                                                ctypes.c_float, ctypes.c_uint64, P, P, P, P,
                                                                ctypes.c_float, ctypes.c_uint64, P]),
    "mapf_conv_nhwc_pool_f16": (ctypes.c_int, [P, P, P, P, I64, I32, I32, I32, I32, I32, I32, P]),
    "mapf_conv_first_f32": (ctypes.c_int, [P, P, P, P, I64, I32, I32, I32, I32, P]),
    "mapf_conv_select": (ctypes.c_int, [I32]),
    "mapf_conv_nhwc_f16": (ctypes.c_int, [P, P, P, P, I64, I32, I32, I32, I32, I32, I32, I32, P]),
    "mapf_attention_f16": (ctypes.c_int, [P, P, P, P, I64, I32, I32, I64, I64, I64, I64, I32, I32, ctypes.c_float, P]),
    "mapf_attention_bwd_f16": (ctypes.c_int, [P, P, P, P, P, P, P, P, I64, I32, I32, I64, I64, I64, I64, I64, I64, I32,
                                              I32, ctypes.c_float, P]),
    "mapf_attention_bwd_select": (ctypes.c_int, [I32]),
}

_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise RuntimeError(f"libmapf.so not found at {LIB_PATH}: build it with `python -c 'import "
                               f"__graft_entry__ as g; g.build()'` (no CPU fallback exists)")
        L = ctypes.CDLL(LIB_PATH)
        for name, (res, args) in SIGNATURES.items():
            fn = getattr(L, name)
            fn.restype = res
            fn.argtypes = args
        if L.mapf_abi_version() != 1:
            raise RuntimeError("libmapf.so ABI mismatch")
        _lib = L
    return _lib


def check(rc):
    if rc != 0:
        msg = lib().mapf_last_error()
        raise RuntimeError(f"libmapf error {rc}: {msg.decode() if msg else ''}")
    return rc
