"""ctypes binding of ``libmlcomp_kernels.so`` (csrc/kernels/*.hip, gfx950).

Every launcher takes raw device pointers plus the current HIP stream of the calling
PyTorch context, so the kernels interleave with (and are captured into HIP graphs
together with) PyTorch's own work.  There is no fallback: on a GPU box a missing or
stale library raises immediately (the driver checks that the native .so is what runs).
"""
from __future__ import annotations

import ctypes as C
import os
import threading

import torch

_LIB = None
_LOCK = threading.Lock()

# Deterministic mode (MLC_DETERMINISTIC=1): every reduction gets one partial-sum copy per
# contributing block (MLC_DET_COPIES of them, default 4096) and split-K GEMMs run unsplit,
# so no two float adds race and a step is bitwise reproducible (graph replay == eager).
# Slower (no split-K) and heavier (bigger reduction scratch): a debugging / testing mode.
DETERMINISTIC = os.environ.get('MLC_DETERMINISTIC', '0') == '1'
# mlc_set_deterministic never uses fewer than the default 32 copies (batchnorm.hip NSTAT), so
# the Python side sizes its reduction buffers with the same floor: fewer would let kernels
# index copies the buffers do not have
DET_COPIES = max(32, int(os.environ.get('MLC_DET_COPIES', '4096')))

vp, i32, i64, f32, u32 = C.c_void_p, C.c_int, C.c_long, C.c_float, C.c_uint

_SIGS = {
    'mlc_conv_fwd': [vp, vp, vp, vp, vp] + [i32] * 12 + [vp, vp, vp],
    'mlc_conv_fwd_ld': [vp, vp, vp] + [i32] * 13 + [vp],
    'mlc_conv_dgrad': [vp] * 4 + [i32] * 12 + [vp] * 11 + [vp],
    'mlc_conv_dgrad_t': [vp] * 4 + [i32] * 12 + [vp] * 11 + [vp],
    'mlc_bilinear_up_fwd': [vp, vp] + [i32] * 6 + [vp],
    'mlc_bilinear_up_bwd': [vp, vp] + [i32] * 6 + [vp],
    'mlc_gn_relu_fwd': [vp, vp, vp, vp, vp] + [i32] * 4 + [f32, vp],
    'mlc_gn_relu_bwd': [vp] * 7 + [i32] * 4 + [f32, vp],
    'mlc_conv_tr_fwd': [vp] * 5 + [i32] * 12 + [vp],
    'mlc_wt_transpose': [vp, i32, i64, vp],
    'mlc_conv_wgrad': [vp, vp, vp] + [i32] * 14 + [vp, i64, vp, vp, vp],
    'mlc_conv_wgrad_native': [vp, vp, vp] + [i32] * 14 + [vp, i64, vp, vp, vp],
    'mlc_gemm_f32out': [vp, vp, vp, vp] + [i32] * 11 + [vp],
    'mlc_gemm_bf16out': [vp, vp, vp] + [i32] * 8 + [vp],
    'mlc_gemm256_nt': [vp, vp, vp, vp] + [i32] * 6 + [vp, i32, vp, vp, i32, i32, vp],
    'mlc_g256_dense': [vp, vp, vp] + [i32] * 7 + [vp, i32, vp, vp, vp, i32, vp],
    'mlc_gemm256_tn': [vp, vp, vp] + [i32] * 8 + [vp],
    'mlc_conv256_fwd': [vp] * 5 + [i32] * 13 + [vp],
    'mlc_augment': [vp, vp, vp, vp] + [i32] * 7 + [vp],
    'mlc_gemm_bf16_ex': [vp, vp, vp] + [i32] * 8 + [vp, i32, vp, vp, vp, vp, i64, vp],
    'mlc_gemm_bf16_ex_native': [vp, vp, vp] + [i32] * 8 + [vp, i32, vp, vp, vp, vp, i64, vp],
    'mlc_ln_fwd': [vp] * 8 + [i32, i32, f32, f32, f32, vp, u32, u32, vp],
    'mlc_ln_bwd': [vp] * 10 + [i32, i32, f32, f32, vp, u32, u32, vp],
    'mlc_ln_finalize_many': [vp, i32, i32, vp],
    'mlc_embed_bwd': [vp] * 7 + [i32] * 4 + [vp],
    'mlc_softmax_fwd': [vp] * 4 + [i64, i32, i32, f32, f32, vp, u32, vp],
    'mlc_softmax_bwd': [vp] * 3 + [i64, i32, f32, f32, vp, u32, vp],
    'mlc_linear_wgrad_bias': [vp] * 4 + [i32] * 7 + [vp, i64, vp],
    'mlc_linear_wgrad_bias_native': [vp] * 4 + [i32] * 7 + [vp, i64, vp],
    # library GEMM selection (blaslt.hip)
    'mlc_blaslt_mode': [i32],
    'mlc_blaslt_choices': [vp, i32],
    'mlc_upcat_fwd': [vp, vp, vp] + [i32] * 5 + [vp],
    'mlc_upcat_bwd': [vp, vp, vp] + [i32] * 5 + [vp],
    'mlc_seg_head_fwd': [vp] * 6 + [i64, i32, i32, vp],
    'mlc_seg_head_bwd': [vp] * 8 + [i64, i32, i32, f32, f32, f32, vp],
    'mlc_attn_fwd': [vp] * 4 + [i32, i32, i32, f32, f32, vp, u32, vp],
    'mlc_attn_bwd': [vp] * 5 + [i32, i32, i32, f32, f32, vp, u32, vp],
    'mlc_flash_fwd': [vp] * 4 + [i32] * 4 + [f32, f32, vp, u32, vp],
    'mlc_flash_bwd': [vp] * 7 + [i32] * 4 + [f32, f32, vp, u32, vp],
    'mlc_flash_bwd128': [i32],
    'mlc_colsum_acc': [vp, vp, vp, i32, i32, vp],
    'mlc_dropout': [vp, vp, i64, f32, vp, u32, vp],
    'mlc_bn_stat_copies': [],
    'mlc_set_deterministic': [i32, i32],
    'mlc_get_stat_copies': [],
    'mlc_get_deterministic': [],
    'mlc_gemm_config': [i32],
    'mlc_gemm_get_set': [i32, i32],
    'mlc_bn_get_set': [i32, i32],
    'mlc_bn_finalize': [vp, vp, i32] + [vp] * 8 + [i64, i32, f32, f32, vp],
    'mlc_bn_fwd_apply': [vp] * 5 + [i64, i32, i32, vp],
    'mlc_bn_fwd_apply2': [vp] * 7 + [i64, i32, i32, vp],
    'mlc_bn_bwd_reduce': [vp] * 5 + [i64, i32, vp],
    'mlc_bn_bwd_finalize': [vp] * 6 + [i64, i32, vp],
    'mlc_bn_fwd_fused': [vp] * 5 + [i32] + [vp] * 10 + [i64, i32, f32, f32, i32, vp],
    'mlc_bn_bwd_fused': [vp] * 5 + [i32] + [vp] * 6 + [i64, i32, vp],
    'mlc_bnact_fused': [vp] * 5 + [i32] + [vp] * 10 + [i64, i32, f32, f32, i32, f32, vp, i64, vp, i32, vp, i64, vp],
    'mlc_bn_bwd_apply': [vp] * 7 + [i64, i32, vp],
    'mlc_maxpool_fwd': [vp, vp, vp] + [i32] * 9 + [vp],
    'mlc_maxpool_bwd': [vp, vp, vp] + [i32] * 9 + [vp],
    'mlc_stem_pool_fwd': [vp] * 6 + [i32] * 4 + [vp],
    'mlc_stem_pool_bwd_reduce_pooled': [vp] * 5 + [i32] * 4 + [vp],
    'mlc_stem_pool_bwd_reduce': [vp] * 5 + [i32] * 4 + [vp],
    'mlc_stem_pool_bwd_apply': [vp] * 6 + [i32] * 4 + [vp],
    'mlc_stem_s2d': [vp, vp] + [i32] * 5 + [vp],
    'mlc_stem_conv_fwd': [vp] * 5 + [i32] * 3 + [vp],
    'mlc_avgpool_fwd': [vp, vp, i32, i32, i32, vp],
    'mlc_avgpool_bwd': [vp, vp, vp, i32, i32, i32, vp],
    'mlc_avgpool2d_fwd': [vp, vp] + [i32] * 10 + [vp],
    'mlc_avgpool2d_bwd': [vp, vp, vp] + [i32] * 10 + [vp],
    'mlc_adaptive_avg_fwd': [vp, vp] + [i32] * 6 + [vp],
    'mlc_adaptive_avg_bwd': [vp, vp] + [i32] * 6 + [vp],
    'mlc_softmax_ce': [vp] * 5 + [i32, i32, i32, f32, f32, vp],
    'mlc_colsum': [vp, vp, i32, i32, vp],
    'mlc_nchw_to_nhwc': [vp, vp, i32, i32, i32, i32, vp],
    'mlc_cast_f32_bf16': [vp, vp, i64, vp],
    'mlc_sgd': [vp] * 5 + [i64, i64, i64, f32, f32, f32, i32, i32, vp],
    'mlc_adam': [vp] * 6 + [i64, i64, i64, f32, f32, f32, f32, i32, vp],
    'mlc_sqnorm': [vp, i64, vp, f32, vp],
    'mlc_opt_config': [i32, i32],
    # generic engine (gconv.hip, normact.hip, igemm.hip extras)
    'mlc_gconv_wb_elems': [i32] * 6,
    'mlc_gconv_fwd': [vp] * 6 + [i32] * 13 + [vp],
    'mlc_gconv_dgrad': [vp] * 4 + [i32] * 13 + [vp],
    'mlc_gconv_wgrad': [vp] * 3 + [i32] * 14 + [vp],
    'mlc_dwconv_fwd': [vp] * 5 + [i32] * 11 + [vp],
    'mlc_dwconv_dgrad': [vp] * 3 + [i32] * 11 + [vp],
    'mlc_dwconv_wgrad': [vp] * 4 + [i32] * 12 + [vp],
    'mlc_bn_stats': [vp, vp, vp, i64, i32, vp],
    'mlc_zero4': [vp, i64, vp, i64, vp, i64, vp, i64, vp],
    'mlc_bn_stats_ld': [vp, vp, vp, i64, i32, i32, i64, vp],
    'mlc_bnact_apply': [vp] * 7 + [i64, i32, i32, f32, vp, i64, vp],
    'mlc_bnact_bwd_reduce': [vp] * 10 + [i64, i32, i32, f32, vp, i64, i64, vp],
    'mlc_bnact_bwd': [vp] * 12 + [i64] + [vp] * 5 + [i64, i32, i32, f32, vp, i64, vp, i64, i64, vp, i32, vp],
    'mlc_bnact_bwd_apply': [vp] * 12 + [i64, i32, i32, f32, vp, i64, vp, i64, i64, vp, i32, vp],
    'mlc_act_fwd': [vp, vp, i64, i32, f32, vp],
    'mlc_act_bwd': [vp] * 4 + [i64, i32, f32, vp],
    'mlc_chscale_fwd': [vp] * 4 + [i32, i64, i32, i32, vp],
    'mlc_chscale_bwd': [vp] * 8 + [i32] * 3 + [vp],
    'mlc_conv_fwd_ex': [vp] * 4 + [i32] * 13 + [vp],
    'mlc_conv_wgrad_bias': [vp] * 4 + [i32] * 13 + [vp, i64, vp],
    'mlc_temporal_unfold': [vp, vp] + [i32] * 9 + [vp],
    'mlc_temporal_fold': [vp, vp, vp] + [i32] * 9 + [vp],
    'mlc_counters_owner': [i32],
    'mlc_counters_release': [i32],
    'mlc_counters_in_use': [],
    'mlc_comm_unique_id_bytes': [],
    'mlc_comm_get_unique_id': [vp],
    'mlc_comm_init': [vp, i32, i32, i32, i32, vp],
    'mlc_comm_async_error': [vp],
    'mlc_comm_abort': [vp],
    'mlc_comm_error_string': [i32],
    'mlc_comm_last_error': [vp],
    'mlc_comm_set_timeout': [i64],
    'mlc_comm_destroy': [vp],
    'mlc_allreduce': [vp, vp, vp, i64, i32, i32, vp],
    'mlc_broadcast': [vp, vp, vp, i64, i32, i32, vp],
    'mlc_reduce_scatter': [vp, vp, vp, i64, i32, i32, vp],
    'mlc_allgather': [vp, vp, vp, i64, i32, vp],
    'mlc_alltoall': [vp, vp, vp, i64, i32, i32, i32, vp],
}
_RESTYPE = {'mlc_comm_init': vp, 'mlc_gconv_wb_elems': C.c_long, 'mlc_counters_owner': None,
            'mlc_counters_release': C.c_long, 'mlc_counters_in_use': C.c_long,
            'mlc_comm_error_string': C.c_char_p, 'mlc_comm_last_error': C.c_char_p, 'mlc_comm_set_timeout': None}


def lib_path():
    """The in-tree kernel library (``MLC_KERNEL_LIB`` points at another build, for A/B runs)."""
    from mlcomp_amd.build import KERNEL_LIB
    return os.environ.get('MLC_KERNEL_LIB') or KERNEL_LIB


def load():
    """Load (building first if absent) the kernel library."""
    global _LIB
    if _LIB is not None:
        return _LIB
    with _LOCK:
        if _LIB is not None:
            return _LIB
        path = lib_path()
        if not os.path.exists(path):
            from mlcomp_amd.build import build_kernels
            build_kernels()
        lib = C.CDLL(path)
        for name, args in _SIGS.items():
            fn = getattr(lib, name)
            fn.argtypes = args
            fn.restype = _RESTYPE.get(name, C.c_int)
        # A/B knobs of the GEMM engine (tile policy / min blocks for the wide-wave tiles)
        for key, env in ((1, 'MLC_SPLIT_TARGET'), (2, 'MLC_SPLIT_TARGET_MAT'), (3, 'MLC_GEMM_BIG'),
                         (4, 'MLC_GEMM_BIG_MIN'), (5, 'MLC_GEMM_SINGLE_STAGE'), (6, 'MLC_SPLITK_FUSED'),
                         (9, 'MLC_SPLIT_TARGET_DENSE'), (12, 'MLC_DENSE_SPLIT_TARGET'), (13, 'MLC_SINGLE_STAGE_KT'),
                         (15, 'MLC_GEMM_PERSIST_NBUF'), (16, 'MLC_GEMM_PERSIST_KT')):
            if os.environ.get(env):
                lib.mlc_gemm_get_set(key, int(os.environ[env]))
        for key, env in ((0, 'MLC_BN_UNROLL'), (1, 'MLC_BN_BLOCKS')):   # BN elementwise passes
            if os.environ.get(env):
                lib.mlc_bn_get_set(key, int(os.environ[env]))
        if DETERMINISTIC:
            lib.mlc_set_deterministic(1, DET_COPIES)
            # torch's own scatter-adds (the BERT embedding gradients) take their
            # deterministic (sort-based) implementations too
            torch.use_deterministic_algorithms(True, warn_only=True)
        _LIB = lib
    return _LIB


def available() -> bool:
    return torch.cuda.is_available()


def stream():
    return C.c_void_p(torch.cuda.current_stream().cuda_stream)


def ptr(t):
    if t is None:
        return None
    return C.c_void_p(t.data_ptr())


def call(name, *args):
    rc = getattr(load(), name)(*args)
    if rc == -2 and DETERMINISTIC:
        raise RuntimeError(f'{name}: deterministic mode needs more partial-sum copies than '
                           f'MLC_DET_COPIES={DET_COPIES} (one per contributing block; raise it)')
    if rc != 0:
        raise RuntimeError(f'{name} failed (rc={rc}); check shape constraints '
                           f'(channels % 8 == 0) or HIP error')
    return rc
