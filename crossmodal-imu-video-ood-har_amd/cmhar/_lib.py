"""ctypes binding of the cmhar C ABI (include/cmhar.h) — the only compute path of this package.

The library is built in-tree (`make -C crossmodal-imu-video-ood-har_amd`, or `__graft_entry__.build()`) as
`cmhar/libcmhar.so`.  There is deliberately NO fallback: if the library is missing or a kernel rejects its
arguments, the call raises.
"""
from __future__ import annotations

import ctypes as C
import os

import torch

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get('CMHAR_LIB', os.path.join(_HERE, 'libcmhar.so'))

F32, BF16, F16 = 0, 1, 2
ACT_NONE, ACT_GELU, ACT_RELU, ACT_DGELU, ACT_DRELU, ACT_GELU_SAVEGRAD, ACT_MULAUX = 0, 1, 2, 3, 4, 5, 6

vp, i32, i64, f32, u64 = C.c_void_p, C.c_int, C.c_long, C.c_float, C.c_ulonglong


class Epilogue(C.Structure):
    _fields_ = [('bias', vp), ('residual', vp), ('ldr', i64), ('aux_in', vp), ('lda', i64), ('aux_out', vp),
                ('ldo', i64), ('rowadd', vp), ('rowadd_mod', i32), ('rowadd_ld', i32), ('act', i32),
                ('alpha', f32), ('beta', f32), ('pdrop', f32), ('pad_', i32), ('seed', u64), ('rowsum', vp),
                ('rowsum_beta', f32), ('colscale_lo', i32), ('colscale_hi', i32), ('colscale', f32)]


class IMULayer(C.Structure):
    """CmharIMULayer (include/cmhar.h): one post-LN encoder layer's parameters and saved activations."""
    _fields_ = ([(n, vp) for n in ('w_qkv', 'b_qkv', 'w_out', 'b_out', 'ln1_g', 'ln1_b', 'w_ff1', 'b_ff1', 'w_ff2',
                                   'b_ff2', 'ln2_g', 'ln2_b')] + [('eps1', f32), ('eps2', f32)] +
                [(n, vp) for n in ('qkv', 'o', 'lse', 's1', 'mu1', 'rs1', 'h1', 'fd', 's2', 'mu2', 'rs2', 'h2')])


class IMULayerGrad(C.Structure):
    """CmharIMULayerGrad (include/cmhar.h): one layer's token-gradient scratch and parameter gradients."""
    _fields_ = [(n, vp) for n in ('dqkv', 'da', 'dpre', 'df2', 'gln1', 'gln2', 'dw_qkv', 'db_qkv', 'dw_out', 'db_out',
                                  'dln1_g', 'dln1_b', 'dw_ff1', 'db_ff1', 'dw_ff2', 'db_ff2', 'dln2_g', 'dln2_b')]


IMU_MAX_LAYERS = 8

_SIGS = {
    'cmhar_version': (i32, []),
    'cmhar_gemm_bf16': (i32, [i32, i32, i32, i32, i32, vp, i64, vp, i64, vp, i64, C.POINTER(Epilogue), i32, vp, vp]),
    'cmhar_gemm_bf16_phased': (i32, [i32, i32, i32, i32, i32, vp, i64, vp, i64, vp, i64, C.POINTER(Epilogue), i32, vp,
                                     vp, i32]),
    'cmhar_gemm_f16': (i32, [i32, i32, i32, i32, i32, vp, i64, vp, i64, vp, i64, C.POINTER(Epilogue), i32, vp, vp]),
    'cmhar_gemm_bf16_ws': (i64, [i32, i32, i32]),
    'cmhar_gemm_bf16_plan': (i32, [i32, i32, i32, i32, i32, i32, i32]),
    'cmhar_gemm_bf16_plan2': (i32, [i32, i32, i32, i32, i32, i32, i32, i32]),
    'cmhar_gemm_generic': (i32, [i32, i32, i32, i32, i32, i32, vp, i64, i64, i64, vp, i64, i64, i64, vp, i64, i64,
                                 C.POINTER(Epilogue), vp]),
    'cmhar_gemm_generic_splitk': (i32, [i32, i32, i32, i32, i32, i32, vp, i64, i64, vp, i64, i64, vp, i64,
                                        C.POINTER(Epilogue), vp, vp]),
    'cmhar_attention_fwd': (i32, [i32, i32, i32, i32, i32, i32, vp, i64, vp, i64, vp, i64, vp, i64, vp, f32, f32, u64,
                                  vp]),
    'cmhar_attention_fwd_opt': (i32, [i32]),
    'cmhar_attention_bwd': (i32, [i32, i32, i32, i32, i32, i32, vp, i64, vp, i64, vp, i64, vp, i64, vp, i64, vp, vp,
                                  vp, i64, vp, i64, vp, i64, f32, f32, u64, vp]),
    'cmhar_attention_bwd_prescaled': (i32, [i32, i32, i32, i32, vp, i64, vp, i64, vp, i64, vp, i64, vp, i64, vp, vp,
                                            vp, i64, vp, i64, vp, i64, f32, vp]),
    'cmhar_layernorm_fwd': (i32, [i32, i32, i32, vp, i64, vp, i64, f32, u64, vp, i64, vp, i64, vp, vp, vp, vp, f32,
                                  vp]),
    'cmhar_layernorm_bwd_ws': (i64, [i32, i32]),
    'cmhar_layernorm_bwd': (i32, [i32, i32, i32, vp, i64, vp, i64, vp, vp, vp, vp, i64, vp, i64, vp, i64, f32, u64,
                                  vp, vp, f32, vp, vp]),
    'cmhar_colsum_ws': (i64, [i32, i32]),
    'cmhar_colsum': (i32, [i32, i32, i32, vp, i64, vp, f32, f32, vp, i64, vp]),
    'cmhar_batchnorm_fwd': (i32, [i32, i32, vp, vp, vp, vp, vp, vp, vp, vp, i32, f32, f32, i32, vp, vp]),
    'cmhar_batchnorm_bwd': (i32, [i32, i32, vp, vp, vp, vp, vp, vp, vp, vp, vp, i32, i32, f32, vp]),
    'cmhar_l2normalize_fwd': (i32, [i32, i32, vp, vp, vp, f32, vp]),
    'cmhar_l2normalize_bwd': (i32, [i32, i32, vp, vp, vp, vp, f32, vp]),
    'cmhar_siglip_ws': (i64, [i32, i32]),
    'cmhar_siglip_loss': (i32, [i32, i32, i32, vp, vp, vp, vp, vp, vp, i32, i32, vp, i32, i32, vp, vp, vp, vp]),
    'cmhar_tubelet_im2col': (i32, [i32, i32, i32, i32, i32, i32, i32, i32, vp, vp, vp]),
    'cmhar_imu_embed_fwd': (i32, [i32, i32, i32, i32, i32, i32, i32, i32, vp, C.POINTER(vp), C.POINTER(vp), vp, vp,
                                  vp, vp]),
    'cmhar_imu_embed_bwd': (i32, [i32, i32, i32, i32, i32, i32, i32, i32, i32, vp, vp, vp, vp, C.POINTER(vp),
                                  C.POINTER(vp), vp]),
    'cmhar_imu_encoder_fwd': (i32, [i32, i32, i32, i32, i32, i32, vp, C.POINTER(IMULayer), vp, vp, f32, vp, vp, vp,
                                    f32, f32, u64, vp]),
    'cmhar_imu_encoder_bwd': (i32, [i32, i32, i32, i32, i32, i32, vp, C.POINTER(IMULayer), C.POINTER(IMULayerGrad),
                                    vp, vp, vp, vp, vp, vp, vp, f32, f32, u64, vp]),
    'cmhar_copy2d': (i32, [i32, i32, i32, i32, vp, i64, vp, i64, f32, f32, f32, u64, vp]),
    'cmhar_logits_energy': (i32, [i32, i32, i32, vp, i64, f32, vp, vp, vp, vp]),
    'cmhar_cross_entropy_ws': (i64, [i32]),
    'cmhar_resize_ksize': (i32, [i32, i32]),
    'cmhar_video_ingest_ws': (i64, [i32, i32, i32, i32, i32]),
    'cmhar_video_ingest': (i32, [i32, i32, vp, i64, i32, i32, vp, i32, i32, vp, vp, i32, vp, vp, i64, vp]),
    'cmhar_imu_preprocess_ws': (i64, [i64, i32, i32]),
    'cmhar_imu_preprocess': (i32, [i32, i32, vp, vp, i64, vp, i32, i32, i64, vp, vp, i32, vp, vp, vp]),
    'cmhar_cross_entropy': (i32, [i32, i32, vp, i64, i64, vp, i64, f32, f32, f32, i32, vp, vp, vp, vp, vp, vp, i64,
                                  i64, f32, f32, vp, vp, vp]),
    'cmhar_mt_grad_norm': (i32, [vp, vp, i32, vp, vp, f32, i32, vp]),
    'cmhar_mt_adamw': (i32, [vp, vp, i32, f32, f32, f32, f32, f32, f32, f32, vp, vp]),
    'cmhar_mt_adamw_clip': (i32, [vp, vp, i32, f32, f32, f32, f32, f32, f32, f32, vp, i32, vp]),
    'cmhar_mt_cast_bf16': (i32, [vp, vp, i32, vp]),
    'cmhar_conv3d_im2col': (i32, [i32, i32, vp, vp, vp, vp]),
    'cmhar_conv3d_col2im': (i32, [i32, vp, vp, vp, i32, vp]),
    'cmhar_conv3d_fwd': (i32, [vp, i32, vp, vp, vp, vp, vp, vp]),
    'cmhar_bn_cl_fwd_tiles': (i32, [i64, i32, i32, vp, vp, vp, vp, vp, vp, vp, vp, vp, vp, f32, f32, i32, vp, vp]),
    'cmhar_conv3d_fwd_tiles': (i32, [vp, i32]),
    'cmhar_conv3d_fwd_split_ws': (i64, [vp, i32]),
    'cmhar_conv3d_fwd_plan': (i32, [vp, i32]),
    'cmhar_conv3d_wgrad_plan': (i32, [vp, i32]),
    'cmhar_conv3d_fwd_split': (i32, [vp, i32, vp, vp, vp, vp, vp, vp]),
    'cmhar_conv3d_stem_tiles': (i32, [vp, i32]),
    'cmhar_conv3d_stem_stats_floats': (i64, [vp, i32]),
    'cmhar_conv_pack_stem': (i32, [i32, i32, i32, i32, i32, vp, vp, vp]),
    'cmhar_conv3d_stem_fwd': (i32, [vp, i32, vp, vp, vp, vp, vp]),
    'cmhar_conv3d_stem_wgrad_ws': (i64, [vp, i32]),
    'cmhar_conv3d_stem_wgrad': (i32, [vp, i32, vp, vp, vp, vp, vp]),
    'cmhar_conv3d_fwd_stats_floats': (i64, [vp, i32]),
    'cmhar_conv3d_wgrad_ws': (i64, [vp, i32]),
    'cmhar_conv3d_wgrad': (i32, [vp, i32, vp, vp, vp, vp, vp]),
    'cmhar_bn_cl_ws': (i64, [i64, i32]),
    'cmhar_bn_cl_fwd': (i32, [i32, i64, i32, vp, vp, vp, vp, vp, vp, vp, vp, vp, i32, f32, f32, i32, vp, vp, vp]),
    'cmhar_bn_cl_bwd': (i32, [i32, i64, i32, vp, vp, vp, vp, vp, vp, vp, vp, vp, vp, i32, i32, vp, vp]),
    'cmhar_bn_cl_bwd_nores': (i32, [i32, i64, i32, vp, vp, vp, vp, vp, vp, vp, vp, vp, i32, i32, vp, vp]),
    'cmhar_avgpool_cl': (i32, [i32, i32, i64, i32, vp, vp, vp]),
    'cmhar_avgpool_cl_bwd': (i32, [i32, i32, i64, i32, vp, vp, vp]),
    'cmhar_video_to_ndhwc': (i32, [i32, i32, i32, i32, i32, i32, vp, vp, vp]),
    'cmhar_conv_pack_weight': (i32, [i32, i32, i32, i32, i32, i32, i32, vp, vp, vp, vp]),
    'cmhar_conv_pack_weights': (i32, [i32, i32, vp, vp, vp]),
    'cmhar_conv_grad_unpack': (i32, [i32, i32, i32, i32, i32, i32, i32, vp, vp, vp]),
    'cmhar_maxpool2d_cl_fwd': (i32, [i32, i32, i32, i32, i32, i32, i32, i32, vp, vp, vp, vp]),
    'cmhar_maxpool2d_cl_bwd': (i32, [i32, i32, i32, i32, i32, i32, i32, i32, vp, vp, vp, vp]),
    'cmhar_dwconv2d_cl_fwd': (i32, [i32, i32, i32, i32, i32, i32, i32, i32, vp, vp, vp, vp]),
    'cmhar_dwconv2d_cl_dgrad': (i32, [i32, i32, i32, i32, i32, i32, i32, i32, vp, vp, vp, vp]),
    'cmhar_dwconv2d_cl_wgrad_ws': (i64, [i32, i32, i32, i32, i32, i32, i32]),
    'cmhar_dwconv2d_cl_wgrad': (i32, [i32, i32, i32, i32, i32, i32, i32, i32, vp, vp, vp, vp, vp]),
    'cmhar_mt_transpose_bf16': (i32, [vp, i32, i32, vp]),
    'cmhar_mfma_peak_probe_flops': (i64, [i32, i32, i32]),
    'cmhar_mfma_peak_probe': (i32, [i32, i32, i32, vp, i32, vp, vp]),
    'cmhar_blaslt_linear': (i32, [i32, i32, i32, i32, vp, i64, vp, i64, vp, i64, vp, vp, i64, vp]),
    'cmhar_blaslt_linear_ok': (i32, [i32, i32, i32, i32, i64, i64, i64, i32, i32, i64]),
}

EXPORTED = tuple(_SIGS)

_lib = None


def lib():
    """Load libcmhar.so (raises if it is missing — there is no fallback path)."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise RuntimeError(f'cmhar HIP library not found at {LIB_PATH}; build it with '
                               f'`make -C crossmodal-imu-video-ood-har_amd` (or __graft_entry__.build())')
        L = C.CDLL(LIB_PATH)
        for name, (res, args) in _SIGS.items():
            fn = getattr(L, name)
            fn.restype = res
            fn.argtypes = args
        _lib = L
    return _lib


def call(name, *args):
    rc = getattr(lib(), name)(*args)
    if rc != 0:
        raise RuntimeError(f'{name} failed with code {rc}')
    return rc


def ptr(t):
    return None if t is None else t.data_ptr()


def stream(device=None):
    return torch.cuda.current_stream(device).cuda_stream


def dtype_code(dt):
    if dt == torch.float32:
        return F32
    if dt == torch.bfloat16:
        return BF16
    if dt == torch.float16:
        return F16
    raise TypeError(f'unsupported dtype {dt}')


class NoReplicate:
    """Mixin of every cmhar module that runs HIP code.  `nn.DataParallel` over more than one device replicates a
    module by shallow-copying it per device (torch `replicate.py`), which would share this package's per-device state
    (packed compute-dtype weight shadows, flat gradient buffers, side streams) between replicas; the copy is refused
    with a pointer to the supported path.  `nn.DataParallel` over ONE device never replicates and works as is."""

    def _replicate_for_data_parallel(self):
        raise RuntimeError(
            f'{type(self).__name__}: nn.DataParallel over several GPUs is not supported by the cmhar HIP modules '
            f'(they keep per-device weight shadows, gradient buffers and streams).  Run one process per GPU with '
            f'cmhar.dist instead (`cmhar.dist.init_from_env()`, `cmhar.dist.GradReducer`, launched by torchrun): it '
            f'keeps DataParallel\'s semantics (global-batch loss, per-replica BatchNorm, summed gradients, device-0 '
            f'running statistics; reference main.py:89-93).')


def epilogue(bias=None, residual=None, aux_in=None, aux_out=None, rowadd=None, rowadd_mod=1, act=ACT_NONE,
             alpha=1.0, beta=0.0, pdrop=0.0, seed=0, rowsum=None, rowsum_beta=0.0, colscale=None):
    """colscale: (lo, hi, s) — columns [lo, hi) multiplied by s before the activation."""
    e = Epilogue()
    if colscale is not None:
        e.colscale_lo, e.colscale_hi, e.colscale = int(colscale[0]), int(colscale[1]), float(colscale[2])
    e.rowsum = ptr(rowsum)
    e.rowsum_beta = rowsum_beta
    e.bias = ptr(bias)
    e.residual = ptr(residual)
    e.ldr = residual.stride(0) if residual is not None else 0
    e.aux_in = ptr(aux_in)
    e.lda = aux_in.stride(0) if aux_in is not None else 0
    e.aux_out = ptr(aux_out)
    e.ldo = aux_out.stride(0) if aux_out is not None else 0
    e.rowadd = ptr(rowadd)
    e.rowadd_mod = rowadd_mod
    e.rowadd_ld = rowadd.stride(0) if rowadd is not None else 0
    e.act = act
    e.alpha = alpha
    e.beta = beta
    e.pdrop = pdrop
    e.seed = seed
    return e
