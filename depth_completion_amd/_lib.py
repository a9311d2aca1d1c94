"""ctypes binding of libdcamd.so (the C ABI in include/dcamd.h).

The library is loaded from the package directory only (in-tree build); there is no fallback:
if it is missing or was built for another ABI, every hot-path entry point raises.
"""
from __future__ import annotations

import ctypes as C
import os
from pathlib import Path

# DC_LIB overrides the in-tree library (A/B experiments between builds); there is still no fallback
_LIB_PATH = Path(os.environ.get("DC_LIB") or Path(__file__).resolve().parent / "libdcamd.so")
ABI_VERSION = 21

vp = C.c_void_p
i32 = C.c_int
i64 = C.c_longlong
f32 = C.c_float
fp = C.POINTER(C.c_float)


class GnTarget(C.Structure):
    """Mirror of ``dc_gn_target`` (include/dcamd.h)."""

    _fields_ = [("acc", vp), ("coff", i32), ("groups", i32), ("cpg", i32), ("hw", i32)]


class GnFuse(C.Structure):
    """Mirror of ``dc_gn_fuse``: GroupNorm statistics fused into a conv epilogue."""

    _fields_ = [
        ("mode", i32), ("nt", i32), ("t", GnTarget * 2),
        ("x", vp), ("x2", vp), ("ldx", i32), ("ldx2", i32), ("c1", i32),
        ("stats", vp), ("gamma", vp), ("beta", vp), ("silu", i32),
    ]


class LnFuse(C.Structure):
    """Mirror of ``dc_ln_fuse``: a LayerNorm of the input rows folded into a linear."""

    _fields_ = [("csum", vp), ("cbias", vp), ("stats", vp)]


class ConvDesc(C.Structure):
    """Mirror of ``dc_conv_desc`` (include/dcamd.h)."""

    _fields_ = [
        ("x", vp), ("x2", vp), ("ldx", i32), ("ldx2", i32), ("c1", i32),
        ("nb", i32), ("hin", i32), ("win", i32), ("cin", i32),
        ("hout", i32), ("wout", i32),
        ("kh", i32), ("kw", i32), ("stride", i32), ("pad", i32), ("mode", i32),
        ("w", vp), ("ktot", i32), ("cout", i32),
        ("bias", vp), ("rowbias", vp), ("rowbias_idx", vp), ("rowbias_ld", i32),
        ("resid", vp), ("ldr", i32), ("mask", vp), ("ldmask", i32), ("act", i32),
        ("y", vp), ("ldy", i32),
        ("ws", vp), ("ws_bytes", i64),
        ("geglu", i32), ("y2", vp), ("ldy2", i32), ("aux", vp), ("ldaux", i32),
        ("algo", i32), ("splitk", i32), ("rows", vp), ("nrows", i32), ("gn", C.POINTER(GnFuse)),
        ("ln", C.POINTER(LnFuse)), ("geglu_n", i32),
    ]


# name -> argtypes (all return int status unless listed in _RESTYPE)
_SIGS = {
    "dc_abi_version": [],
    "dc_build_id": [],
    "dc_conv_num_algos": [],
    "dc_conv_gemm": [C.POINTER(ConvDesc), vp],
    "dc_groupnorm_ws_bytes": [i32, i32, i32, i32],
    "dc_groupnorm_fwd": [vp, i32, vp, i32, i32, i32, i32, i32, i32, f32, vp, vp, i32, vp, i32, vp, vp, vp],
    "dc_groupnorm_bwd": [vp, i32, vp, i32, i32, i32, i32, i32, i32, vp, vp, i32, vp, vp, i32, vp, i32, vp, i32,
                         vp, i32, vp, vp],
    "dc_gn_acc_bytes": [i32, i32],
    "dc_gn_fuse_pays": [i32, i32, i32, i32],
    "dc_groupnorm_fwd_acc": [vp, i32, vp, i32, i32, i32, i32, i32, i32, f32, vp, vp, i32, vp, vp, i32, vp, vp],
    "dc_groupnorm_bwd_acc": [vp, i32, vp, i32, i32, i32, i32, i32, i32, vp, vp, vp, vp, i32, vp, i32, vp, i32,
                             vp, i32, vp],
    "dc_layernorm_fwd": [vp, i32, i64, i32, f32, vp, vp, vp, i32, vp, vp],
    "dc_layernorm_bwd": [vp, i32, i64, i32, vp, vp, vp, i32, vp, i32, vp, i32, vp],
    "dc_attn_fwd": [vp, i32, i32, i32, i32, vp, i32, vp, vp, i64, vp],
    "dc_attn_bwd": [vp, i32, vp, i32, vp, i32, vp, i32, i32, i32, vp, vp, i32, vp, i64, vp],
    "dc_crossattn_tables_bytes": [i32, i32],
    "dc_crossattn_prepare": [vp, vp, i32, i32, vp, vp],
    "dc_crossattn_fwd": [vp, i32, i64, i32, i32, f32, vp, vp, vp, vp, vp, i32, vp, vp, vp, f32, vp],
    "dc_crossattn_bwd": [vp, i32, i64, i32, i32, vp, vp, vp, vp, vp, i32, vp, i32, vp],
    "dc_crossattn_bwd_ln": [vp, i32, i64, i32, i32, vp, vp, vp, vp, vp, i32, vp, i32, vp, vp, i32, vp, i32, vp],
    "dc_geglu_fwd": [vp, i32, i64, i32, vp, i32, vp],
    "dc_geglu_bwd": [vp, i32, i64, i32, vp, i32, vp, i32, vp],
    "dc_upsample_adjoint": [vp, i32, i32, i32, i32, i32, i32, i32, vp, i32, vp, i32, vp],
    "dc_taesd_clamp_fwd": [vp, i32, i64, vp, vp],
    "dc_taesd_clamp_bwd": [vp, i32, vp, i32, i64, vp, vp, vp, vp, vp],
    "dc_silu": [vp, i64, vp, vp],
    "dc_preprocess_image": [vp, i32, i32, i32, i32, i32, i32, i32, i32, vp, vp],
    "dc_nhwc_to_nchw": [vp, i32, i32, i64, i32, vp, vp],
    "dc_nchw_to_nhwc": [vp, i32, i64, i32, vp, i32, vp],
    "dc_sparse_setup": [vp, i32, i32, i32, i32, f32, f32, vp, i32, i32, i32, vp, vp, vp, vp, vp],
    "dc_preview": [vp, vp, i32, i32, vp, vp, vp, vp, vp, vp],
    "dc_sparse_loss": [vp, i32, i32, i32, i32, i32, i32, i32, i32, vp, vp, vp, vp, vp, vp, vp, vp, vp],
    "dc_decode_tail_bwd": [vp, i32, vp, i32, i32, i32, i32, i32, vp, vp],
    "dc_latent_update": [vp, vp, vp, vp, i32, i32, vp, vp, vp, vp, vp, vp, vp, vp, vp, vp, vp, i32, i32, f32, vp, i64,
                         vp],
    "dc_step_advance": [vp, i32, vp],
    "dc_latent_init": [vp, i32, vp, f32, i32, i32, vp, vp],
    "dc_final_dense": [vp, i32, i32, i32, i32, i32, i32, i32, i32, vp, vp, i32, vp, vp],
    "dc_ddim_step": [vp, vp, i32, i32, vp, vp, vp],
    "dc_closed_form_affine": [vp, i32, i32, i32, i32, i32, i32, i32, i32, vp, vp, vp, vp, vp, vp],
    "dc_sparse_loss_cf": [vp, i32, i32, i32, i32, i32, i32, i32, i32, vp, vp, vp, vp, vp, vp, vp],
    "dc_affine_fit": [vp, i32, i32, i32, i32, i32, i32, i32, i32, vp, vp, vp, vp, i32, f32, i32, vp, vp, vp],
    "dc_dense_loss_ws_bytes": [i32, i32, i32],
    "dc_guide_map": [vp, vp, vp, i32, i32, i32, vp, vp],
    "dc_dense_loss": [vp, i32, i32, i32, i32, i32, i32, i32, i32, vp, vp, vp, vp, vp, i32, vp, vp, vp, vp, vp],
    "dc_closed_form_stats": [vp, i32, i32, i32, i32, i32, i32, i32, i32, vp, vp, vp, vp, vp, vp],
    "dc_closed_form_adjoint": [vp, i32, i32, i32, i32, i32, i32, i32, i32, vp, vp, vp, vp, vp, vp, vp, vp],
    "dc_affine_step": [i32, vp, i32, f32, i32, vp, vp, vp],
    "dc_tap_mask": [vp, vp, vp, i32, i32, i32, i32, i32, i32, i32, vp, vp],
    "dc_dilate_mask": [vp, i32, i32, i32, vp, vp],
    "dc_mask_rows_ws_bytes": [i64],
    "dc_mask_count": [vp, i64, vp, vp, vp],
    "dc_mask_rows": [vp, i64, vp, vp, i32, vp, vp],
    "dc_pad_rows": [vp, vp, i32, vp],
    "dc_memset_async": [vp, i32, i64, vp],
    "dc_latent_scale_fwd": [vp, i32, i64, f32, vp, vp],
    "dc_latent_scale_bwd": [vp, i32, i64, f32, vp, vp, vp, vp, vp],
    "dc_softmax_rows": [vp, i32, i64, i32, f32, vp, i32, vp],
    "dc_softmax_rows_bwd": [vp, i32, vp, i32, i64, i32, f32, vp, i32, vp],
    "dc_transpose": [vp, i32, i32, i32, vp, i32, vp],
    "dc_depth_metrics_ws_bytes": [],
    "dc_depth_metrics": [vp, vp, i64, f32, f32, vp, i32, vp, vp, vp],
    "dc_ensemble_ws_bytes": [i32, i64],
    "dc_ensemble_fit": [vp, i32, i32, i64, vp, vp, vp, vp, i64, vp],
}
_SIGS.update({
    "dc_schedule_tables": [i32, C.c_double, C.c_double, i32, vp, vp, vp],
    "dc_timestep_embedding": [vp, i32, i32, vp],
    "dc_fold_cross_attention": [vp, vp, vp, vp, vp, vp, i32, i32, i32, i32, i32, i32, vp, vp, vp],
    "dc_fold_linear_pair": [vp, vp, i32, i32, vp, vp, vp, vp, vp],
    "dc_fold_layernorm": [vp, i32, i32, vp, vp, vp, vp, vp, vp],
    "dc_conv_pick": [vp, vp, i32, vp, vp],
    "dc_sample_params_default": [vp],
    "dc_latent_hw": [i32, i32, i32, vp, vp],
    "dc_create": [vp, i32],
    "dc_destroy": [vp],
    "dc_session_error": [vp],
    "dc_load_weights": [vp, C.c_char_p, C.c_char_p],
    "dc_encode": [vp, vp, i32, i32, i32, i32, vp, vp],
    "dc_guided_sample": [vp, vp, vp, i32, vp, vp, i32, i32, i32, vp, vp, vp, vp],
    "dc_decode_dense": [vp, vp, vp, vp, i32, i32, i32, vp, vp, vp],
    "dc_complete": [vp, vp, vp, i32, i32, i32, vp, i32, vp, vp, vp, vp, vp],
})
_RESTYPE = {"dc_session_error": C.c_char_p, "dc_sample_params_default": None,
            "dc_build_id": C.c_char_p, "dc_mask_rows_ws_bytes": i64, "dc_groupnorm_ws_bytes": i64, "dc_gn_acc_bytes": i64, "dc_dense_loss_ws_bytes": i64, "dc_depth_metrics_ws_bytes": i64,
             "dc_ensemble_ws_bytes": i64, "dc_crossattn_tables_bytes": i64}

STATUS = {0: "ok", 1: "invalid argument / shape", 2: "kernel launch failed", 3: "alignment contract violated"}


class DCError(RuntimeError):
    pass


_lib = None


def lib_path() -> Path:
    return _LIB_PATH


def load():
    """Load libdcamd.so once; raises if it is absent (no CPU fallback exists)."""
    global _lib
    if _lib is not None:
        return _lib
    if not _LIB_PATH.exists():
        raise DCError(f"{_LIB_PATH} not found: build it with `python -m depth_completion_amd.build` "
                      "(the HIP extension is required; there is no fallback path)")
    lib = C.CDLL(str(_LIB_PATH))
    for name, args in _SIGS.items():
        fn = getattr(lib, name)
        fn.argtypes = args
        fn.restype = _RESTYPE.get(name, i32)
    if lib.dc_abi_version() != ABI_VERSION:
        raise DCError(f"libdcamd ABI {lib.dc_abi_version()} != expected {ABI_VERSION}; rebuild")
    check_provenance(lib)
    _lib = lib
    return lib


def build_id(lib=None) -> str:
    return (lib or load()).dc_build_id().decode()


def check_provenance(lib) -> None:
    """Refuse a library whose build id differs from the hash of the sources in this tree (a stale or foreign
    binary); DC_LIB (an explicit A/B library) skips the check, as does a tree shipped without sources."""
    if os.environ.get("DC_LIB"):
        return
    from . import build as _build
    if not all(f.exists() for f in _build.source_files()):
        return
    want, have = _build.source_hash(), lib.dc_build_id().decode()
    if want != have:
        raise DCError(f"{_LIB_PATH} was built from other sources (build id {have}, tree {want}): rebuild it with "
                      "`python -m depth_completion_amd.build`")


def exported_symbols() -> list[str]:
    return list(_SIGS)


def check(status: int, name: str):
    if status != 0:
        raise DCError(f"{name} failed: {STATUS.get(status, status)}")


def call(name: str, *args):
    st = getattr(load(), name)(*args)
    check(st, name)
