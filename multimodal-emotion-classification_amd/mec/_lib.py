"""ctypes binding of libmec_hip.so (the C ABI declared in include/mec.h).

The library is built in-tree by __graft_entry__.build() (csrc/Makefile). There is no
fallback: if the library or a GPU is missing, load() raises MecError.
"""
import ctypes
import os
import threading

_HERE = os.path.dirname(os.path.abspath(__file__))
# MEC_LIB selects another build of the same ABI (tools/ only: libmec_hip_probes.so, the
# -DMEC_PROBES build whose probe option values return wrong results).
LIB_PATH = os.environ.get('MEC_LIB') or os.path.join(_HERE, 'libmec_hip.so')
PROBES_LIB_PATH = os.path.join(_HERE, 'libmec_hip_probes.so')

c_vp = ctypes.c_void_p
c_int = ctypes.c_int
c_fp = ctypes.POINTER(ctypes.c_float)
c_dp = ctypes.POINTER(ctypes.c_double)

# name -> (restype, argtypes); mirrors include/mec.h one to one.
SIGNATURES = {
    'mec_version': (ctypes.c_char_p, []),
    'mec_last_error': (ctypes.c_char_p, []),
    'mec_blob_size': (ctypes.c_longlong, [c_int]),
    'mec_create': (c_int, [c_int, c_fp, ctypes.c_size_t, c_int, ctypes.POINTER(c_vp)]),
    'mec_create_ex': (c_int, [c_int, c_fp, ctypes.c_size_t, c_int, c_int, ctypes.POINTER(c_vp)]),
    'mec_create_opt': (c_int, [c_int, c_fp, ctypes.c_size_t, c_int, c_int, ctypes.c_char_p, ctypes.POINTER(c_vp)]),
    'mec_model_x3_report': (ctypes.c_char_p, [c_vp]),
    'mec_precision': (c_int, [c_vp]),
    'mec_destroy': (c_int, [c_vp]),
    'mec_speech_fwd': (c_int, [c_vp, c_vp, c_int, c_vp, c_vp, c_vp, c_vp]),
    'mec_text_fwd': (c_int, [c_vp, c_vp, c_vp, c_int, c_int, c_vp, c_vp, c_vp, c_vp]),
    'mec_image_fwd': (c_int, [c_vp, c_vp, c_int, c_vp, c_vp, c_vp, c_vp]),
    'mec_image_fwd_u8': (c_int, [c_vp, c_vp, c_int, c_int, c_int, c_int, c_vp, c_vp, c_vp, c_vp]),
    'mec_fusion_fwd': (c_int, [c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_int, c_vp, c_vp, c_vp, c_vp, c_vp]),
    'mec_audio_fwd': (c_int, [c_vp, c_vp, c_int, c_int, c_vp, c_vp, c_vp]),
    'mec_fuse_weighted': (c_int, [c_vp, c_vp, c_vp, c_int, c_vp, c_vp]),
    'mec_fuse_weighted_f64': (c_int, [c_vp, c_vp, c_vp, c_int, c_vp, c_vp]),
    'mec_resize_u8': (c_int, [c_vp, c_int, c_int, c_int, c_vp, c_int, c_int, c_vp]),
    'mec_gemm_f16': (c_int, [c_vp, c_vp, c_vp, c_vp, c_int, c_vp, c_vp, c_int, c_int, c_int, c_int, c_vp]),
    'mec_gemm_f16x3': (c_int, [c_vp, ctypes.c_longlong, c_vp, ctypes.c_longlong, ctypes.c_float, c_vp, c_vp, c_vp,
                               ctypes.c_longlong, c_vp, c_int, c_int, c_int, c_int, c_vp]),
    'mec_conv_f16': (c_int, [c_vp, c_vp, c_vp, c_vp, c_vp, c_int, c_int, c_int, c_int, c_int, c_int, c_int,
                             c_int, c_int, c_vp]),
    'mec_gemm_f32': (c_int, [c_vp, c_vp, c_vp, c_vp, c_vp, c_int, c_int, c_int, c_int, c_vp]),
    'mec_conv_f32': (c_int, [c_vp, c_vp, c_vp, c_vp, c_vp, c_int, c_int, c_int, c_int, c_int, c_int, c_int,
                             c_int, c_int, c_vp]),
    'mec_set_option': (c_int, [ctypes.c_char_p, c_int]),
    'mec_model_set_option': (c_int, [c_vp, ctypes.c_char_p, c_int]),
    'mec_build_flags': (c_int, []),
    'mec_model_gemm_query': (c_int, [c_vp, c_int, c_int, c_int, c_int]),
    'mec_gemm_query': (c_int, [c_int, c_int, c_int, c_int]),
    'mec_gemm_f32_query': (c_int, [c_int, c_int, c_int, c_int]),
    'mec_model_check': (c_int, [c_vp]),
    'mec_prof_enable': (c_int, [c_vp, c_int]),
    'mec_prof_read': (c_int, [c_vp, c_dp, ctypes.POINTER(c_int)]),
}

# Kernel tags for mec_prof_enable (csrc/mec_common.h KernelTag).
TAGS = {'bert_qkv': 1, 'bert_attn': 2, 'bert_oproj': 3, 'bert_ffn1': 4, 'bert_ffn2': 5, 'bert_ln': 6,
        'resnet_conv3x3': 7, 'resnet_conv1x1': 8, 'resnet_stem': 9, 'speech': 10, 'fusion': 11,
        'mbv2_blocks': 12, 'mbv2_last': 13, 'audio': 14}


# Handle precision (include/mec.h MEC_PREC_*): 'f16' = f16 MFMA operands with fp32
# accumulation / LayerNorm / softmax / residual (the fast path), 'fp32' = fp32 throughout,
# 'fp32x3' = the fp32 path with its GEMM operands as exact f16 hi/lo pairs on the f16 MFMA.
PRECISIONS = {'f16': 0, 'fp32': 1, 'fp32x3': 2}


# mec_model_check's return code for a raised fp32x3 range flag (include/mec.h MEC_ERR_X3_RANGE)
ERR_X3_RANGE = -2


class MecError(RuntimeError):
    pass


class X3RangeError(MecError):
    """An fp32x3 handle's activation planes left the f16 range (mec_model_check == MEC_ERR_X3_RANGE):
    the batch's outputs are invalid; it can be re-run on an fp32 handle of the same weights."""


_lib = None
_lock = threading.Lock()


def load(path: str = LIB_PATH):
    """Load and declare the library (no GPU needed to load it)."""
    global _lib
    with _lock:
        if _lib is not None and path == LIB_PATH:
            return _lib
        if not os.path.exists(path):
            raise MecError(f'{path} is missing: build it with `python -c "import __graft_entry__ as g; g.build()"`')
        lib = ctypes.CDLL(path)
        for name, (res, args) in SIGNATURES.items():
            fn = getattr(lib, name)
            fn.restype = res
            fn.argtypes = args
        if path == LIB_PATH:
            _lib = lib
        return lib


def check(rc: int, what: str):
    if rc != 0:
        err = load().mec_last_error()
        raise (X3RangeError if rc == ERR_X3_RANGE else MecError)(
            f'{what} failed: {err.decode() if err else "unknown error"}')
