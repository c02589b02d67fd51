"""ctypes bindings to the in-tree native libraries.

``libddl_kernels.so`` holds every HIP/CDNA4 kernel of the framework (built by
:mod:`ddl25spring_amd._build` with ``hipcc --offload-arch=gfx950``); ``libddl_runtime.so`` the
host-side C++ runtime (schedules, epoch planner, bucket planner).

Policy: on a machine with a GPU the HIP library is *required* — every op raises if it is missing
or fails to load, there is no silent fallback to PyTorch kernels. CPU tensors (unit tests, the
gloo-only configs) go through the pure-PyTorch reference implementations in
:mod:`ddl25spring_amd.ops.reference`.
"""
from __future__ import annotations

import ctypes
import os
from pathlib import Path

import torch

LIBDIR = Path(__file__).resolve().parent.parent / "lib"
# DDL_KERNEL_LIB: an alternative build of the kernel library (A/B timing of two builds)
KERNEL_LIB_PATH = Path(os.environ["DDL_KERNEL_LIB"]) if os.environ.get("DDL_KERNEL_LIB") else \
    LIBDIR / "libddl_kernels.so"
RUNTIME_LIB_PATH = LIBDIR / "libddl_runtime.so"

_kernels = None
_runtime = None

vp = ctypes.c_void_p
i32 = ctypes.c_int
i64 = ctypes.c_longlong
u64 = ctypes.c_ulonglong
f32 = ctypes.c_float
fp = ctypes.POINTER(ctypes.c_float)


class ConvArgs(ctypes.Structure):
    _fields_ = [("x", vp), ("w", vp), ("dy", vp), ("out", vp), ("stats", vp), ("bias", vp),
                ("residual", vp), ("mask", vp), ("zero", vp),
                ("x_gs", i64), ("w_gs", i64), ("dy_gs", i64), ("out_gs", i64), ("bias_gs", i64),
                ("stats_gs", i64),
                ("G", i32), ("N", i32), ("H", i32), ("W", i32), ("C", i32), ("K", i32), ("R", i32),
                ("S", i32), ("P", i32), ("Q", i32), ("stride", i32), ("pad", i32),
                ("relu", i32), ("accumulate", i32), ("split_k", i32), ("stats_stripes", i32),
                ("bn_x", vp), ("bn_mean", vp), ("bn_rstd", vp), ("partial", vp), ("partial_cap", i64),
                ("mask_scale", vp), ("mask_shift", vp), ("res_gs", i64), ("res_sub", i32), ("gscale", f32)]


class BNArgs(ctypes.Structure):
    _fields_ = [("stats", vp), ("gamma", vp), ("beta", vp), ("running_mean", vp),
                ("running_var", vp), ("scale", vp), ("shift", vp), ("mean", vp), ("rstd", vp),
                ("gs_param", i64), ("gs_buf", i64), ("G", i32), ("C", i32), ("count", i64),
                ("eps", f32), ("momentum", f32), ("training", i32), ("stripes", i32)]


class BNFArgs(ctypes.Structure):  # bn_f32.hip: BNArgs + the per-tile centred-statistics row count
    _fields_ = BNArgs._fields_ + [("tile_rows", i32), ("pad_", i32)]


class BNBwdArgs(ctypes.Structure):
    _fields_ = [("x", vp), ("mean", vp), ("rstd", vp), ("gamma", vp), ("dgamma", vp), ("dbeta", vp),
                ("part", vp), ("coef", vp), ("dx", vp), ("gs_param", i64)]


class HeadArgs(ctypes.Structure):
    _fields_ = [("x", vp), ("w", vp), ("b", vp), ("labels", vp), ("loss", vp), ("correct", vp),
                ("dw", vp), ("db", vp), ("dx", vp), ("c", vp), ("mean", vp), ("rstd", vp), ("part", vp),
                ("pooled", vp), ("dlog", vp),
                ("w_gs", i64), ("b_gs", i64), ("dw_gs", i64), ("db_gs", i64), ("G", i32), ("N", i32),
                ("HW", i32), ("C", i32), ("ncls", i32), ("S", i32), ("scale", f32)]


class ConvF32Args(ctypes.Structure):  # conv_f32.hip
    _fields_ = [("x", vp), ("w", vp), ("dy", vp), ("out", vp), ("stats", vp), ("bias", vp), ("residual", vp),
                ("mask", vp), ("in_scale", vp), ("in_shift", vp), ("bn_x", vp), ("bn_mean", vp), ("bn_rstd", vp),
                ("mask_scale", vp), ("mask_shift", vp), ("partial", vp), ("partial_cap", i64),
                ("x_gs", i64), ("w_gs", i64), ("dy_gs", i64), ("out_gs", i64), ("bias_gs", i64), ("res_gs", i64),
                ("G", i32), ("N", i32), ("H", i32), ("W", i32), ("C", i32), ("K", i32), ("R", i32), ("S", i32),
                ("P", i32), ("Q", i32), ("stride", i32), ("pad", i32), ("relu", i32), ("accumulate", i32),
                ("split_k", i32), ("res_sub", i32), ("in_relu", i32), ("slots", i32), ("gscale", f32),
                ("wsplit", vp), ("ws_gs", i64), ("dyb_x", vp), ("dyb_coef", vp), ("dyb_out", vp),
                ("tickets", vp), ("tickets_cap", i64)]


class BNFBwdArgs(ctypes.Structure):  # bn_f32.hip
    _fields_ = [("x", vp), ("mean", vp), ("rstd", vp), ("gamma", vp), ("dgamma", vp), ("dbeta", vp),
                ("part", vp), ("coef", vp), ("dx", vp), ("gs_param", i64), ("slots", i32), ("pad0_", i32),
                ("fold_ws", vp), ("tickets", vp)]


class HeadFArgs(ctypes.Structure):  # bn_f32.hip
    _fields_ = [("x", vp), ("w", vp), ("b", vp), ("labels", vp), ("loss", vp), ("correct", vp),
                ("dw", vp), ("db", vp), ("dx", vp), ("c", vp), ("mean", vp), ("rstd", vp), ("part", vp),
                ("pooled", vp), ("dlog", vp), ("row_loss", vp), ("row_hit", vp),
                ("w_gs", i64), ("b_gs", i64), ("dw_gs", i64), ("db_gs", i64), ("G", i32), ("N", i32),
                ("HW", i32), ("C", i32), ("ncls", i32), ("scale", f32)]


class SGDArgs(ctypes.Structure):
    _fields_ = [("p", vp), ("g", vp), ("mom", vp), ("shadow", vp), ("n", i64), ("lr", f32),
                ("wd", f32), ("momentum", f32), ("dampening", f32), ("grad_scale", f32),
                ("nesterov", i32), ("first_step", i32)]


class SGDDirectArgs(ctypes.Structure):
    _fields_ = [("p", vp), ("g", vp), ("shadow", vp), ("dmap", vp), ("rows", i64), ("P", i64),
                ("lr", f32), ("grad_scale", f32)]


class AdamArgs(ctypes.Structure):
    _fields_ = [("p", vp), ("g", vp), ("m", vp), ("v", vp), ("shadow", vp), ("n", i64),
                ("lr", f32), ("beta1", f32), ("beta2", f32), ("eps", f32), ("wd", f32),
                ("grad_scale", f32), ("bc1", f32), ("bc2", f32), ("decoupled", i32),
                ("amsgrad_unused", i32), ("step_dev", vp), ("row_len", i64)]


_SIGS = {
    # conv_igemm.hip
    "ddl_conv_fwd": [ctypes.POINTER(ConvArgs), i32, vp],
    "ddl_conv_dgrad": [ctypes.POINTER(ConvArgs), i32, vp],
    "ddl_conv_wgrad": [ctypes.POINTER(ConvArgs), i32, vp],
    "ddl_conv_pair": [ctypes.POINTER(ConvArgs), i32, i32, ctypes.POINTER(ConvArgs), i32, i32, vp],
    "ddl_conv_pair_supported": [ctypes.POINTER(ConvArgs), i32, i32, ctypes.POINTER(ConvArgs), i32, i32],
    # batchnorm.hip
    "ddl_bn_finalize": [ctypes.POINTER(BNArgs), vp],
    "ddl_bn_apply": [vp, vp, vp, vp, vp, vp, vp, i64, i32, i32, i32, vp],
    "ddl_bn_bwd_reduce": [vp, vp, vp, vp, vp, vp, vp, vp, vp, i64, i64, i32, i32, vp],
    "ddl_bn_bwd_apply": [vp, vp, vp, vp, vp, vp, i64, vp, vp, vp, vp, i64, i32, i32, vp],
    "ddl_bn_stats": [vp, vp, i64, i32, i32, vp],
    "ddl_bn_backward": [vp, vp, vp, vp, vp, vp, i64, vp, vp, vp, vp, vp, vp, i64, i32, i32, i32, vp],
    "ddl_bn_finalize2": [ctypes.POINTER(BNArgs), ctypes.POINTER(BNArgs), vp],
    "ddl_bn_backward2": [vp, ctypes.POINTER(BNBwdArgs), ctypes.POINTER(BNBwdArgs), i64, i32, i32, vp],
    "ddl_bn_bwd_reduce_part": [vp, vp, vp, vp, vp, vp, i64, i32, i32, vp],
    # nn_ops.hip
    "ddl_prep_images": [vp, vp, vp, vp, vp, i32, i32, i32, i32, i32, i32, i32, i32, vp, vp, vp],
    "ddl_nchw_to_nhwc": [vp, vp, i32, i32, i32, i32, i32, i32, i32, i32, vp],
    "ddl_maxpool_fwd": [vp, vp, vp, i32, i32, i32, i32, i32, i32, i32, vp],
    "ddl_maxpool_bwd": [vp, vp, vp, vp, i32, i32, i32, i32, i32, i32, i32, vp],
    "ddl_maxpool2_fwd": [vp, vp, i32, i32, i32, i32, vp],
    "ddl_maxpool2_bwd": [vp, vp, vp, i32, i32, i32, i32, vp],
    "ddl_avgpool_fwd": [vp, vp, i32, i32, i32, vp],
    "ddl_avgpool_bwd": [vp, vp, i32, i32, i32, vp],
    "ddl_avgpool_bwd_bn": [vp, vp, vp, vp, vp, vp, vp, i32, i32, i32, i32, vp],
    "ddl_dropout": [vp, vp, i64, f32, u64, u64, vp, vp],
    "ddl_u64_add": [vp, u64, vp],
    "ddl_act_fwd": [vp, vp, i64, i32, f32, vp],
    "ddl_act_bwd": [vp, vp, vp, i64, i32, f32, vp],
    "ddl_channel_sum": [vp, vp, i64, i64, i32, i32, vp],
    "ddl_cast_f32_bf16": [vp, vp, i64, vp],
    "ddl_cast_bf16_f32": [vp, vp, i64, vp],
    # loss.hip
    "ddl_ce_fwd_bwd": [vp, vp, vp, i32, i32, i32, i32, f32, vp, vp, vp, vp],
    "ddl_ce_vocab": [vp, vp, i32, i32, i32, f32, i32, vp, vp, vp],
    "ddl_mse_kl": [vp, vp, i64, vp, vp, i64, f32, f32, vp, vp, vp, vp, vp],
    "ddl_bce_logits": [vp, i32, vp, f32, i32, f32, vp, vp, vp],
    "ddl_head_train": [ctypes.POINTER(HeadArgs), vp],
    # optim.hip
    "ddl_sgd": [ctypes.POINTER(SGDArgs), vp],
    "ddl_sgd_direct": [ctypes.POINTER(SGDDirectArgs), vp],
    "ddl_adam": [ctypes.POINTER(AdamArgs), vp],
    # aggregate.hip
    "ddl_weighted_sum": [vp, i64, vp, i32, i64, vp, i32, vp],
    "ddl_broadcast_rows": [vp, vp, i64, i32, i64, vp, i64, vp],
    "ddl_gram_f32": [vp, i64, vp, i32, i64, vp, i64, vp, vp],
    "ddl_gram_f32_workspace": [i32, i64],
    "ddl_gemm_nt_bf16": [vp, vp, vp, i32, i32, i32, i64, vp],
    "ddl_coord_select": [vp, i64, i32, i64, i32, i32, vp, vp],
    "ddl_pack_shards": [vp, i64, i32, i64, i32, i64, i32, vp, vp],
    "ddl_krum_select": [vp, i32, i32, i32, vp, vp, vp, vp],
    "ddl_mean_rows_idx": [vp, i64, vp, i32, i64, vp, vp],
}

# fp32-activation twins of the templated memory-bound launchers (nn_ops.hip): same signatures
for _n in ("ddl_prep_images", "ddl_nchw_to_nhwc", "ddl_maxpool_fwd", "ddl_maxpool_bwd", "ddl_maxpool2_fwd",
           "ddl_maxpool2_bwd", "ddl_avgpool_fwd", "ddl_avgpool_bwd", "ddl_dropout", "ddl_act_fwd", "ddl_act_bwd",
           "ddl_channel_sum", "ddl_ce_fwd_bwd"):
    _SIGS[_n + "_f32"] = _SIGS[_n]
_SIGS.update({
    # conv_f32.hip
    "ddl_convf32": [ctypes.POINTER(ConvF32Args), i32, i32, vp],
    "ddl_convf32_slots": [ctypes.POINTER(ConvF32Args), i32, i32],
    "ddl_convf32_workspace": [ctypes.POINTER(ConvF32Args), i32, i32],
    # conv_x6h.hip
    "ddl_x6h": [ctypes.POINTER(ConvF32Args), i32, i32, vp],
    "ddl_x6h_ok": [ctypes.POINTER(ConvF32Args), i32, i32],
    "ddl_x6h_slots": [ctypes.POINTER(ConvF32Args), i32],
    "ddl_x6hw": [ctypes.POINTER(ConvF32Args), vp],
    "ddl_x6hw_ok": [ctypes.POINTER(ConvF32Args)],
    "ddl_x6hw_tiles": [ctypes.POINTER(ConvF32Args)],
    "ddl_convf32_wgrad_reduce": [vp, vp, i64, i32, i64, i32, i32, f32, vp],
    "ddl_x6h_workspace": [ctypes.POINTER(ConvF32Args), i32, i32],
    "ddl_x6_split_weights": [vp, vp, i32, i32, i32, i32, i32, i64, i64, i32, vp],
    "ddl_x6_split_weights_multi": [vp, i32, i32, vp],
    "ddl_bce_logits_f32": [vp, i32, vp, f32, i32, f32, vp, vp, vp],
    "ddl_gan_inputs": [vp, i32, i32, i32, i32, vp, vp, vp],
    "ddl_x6_split_desc_size": [],
    # bn_f32.hip
    "ddl_bnf_finalize": [ctypes.POINTER(BNFArgs), ctypes.POINTER(BNFArgs), vp],
    "ddl_bnf_apply": [vp, vp, vp, vp, vp, vp, vp, i64, i32, i32, i32, vp],
    "ddl_bnf_reduce_slots": [i64, i32, i32],
    "ddl_bnf_reduce": [vp, vp, vp, vp, vp, vp, i64, i32, i32, vp],
    "ddl_bnf_stats": [vp, vp, i64, i32, i32, vp],
    "ddl_bnf_backward": [vp, vp, ctypes.POINTER(BNFBwdArgs), ctypes.POINTER(BNFBwdArgs), vp, i64, i32, i32, i32, vp],
    "ddl_avgpoolf_bwd_bn": [vp, vp, vp, vp, vp, vp, vp, i32, i32, i32, i32, vp],
    "ddl_headf_train": [ctypes.POINTER(HeadFArgs), vp],
    "ddl_bnf_channel_sum": [vp, vp, i64, vp, i64, i32, i32, vp],
    "ddl_bnf_fold_ws": [i32, i32, i32],
    "ddl_bnf_fold_tickets": [i32, i32],
    "ddl_bnf_coef_apply": [vp, vp, vp, vp, i64, i32, i32, vp],
})
_RESTYPES = {"ddl_convf32_slots": ctypes.c_longlong, "ddl_convf32_workspace": ctypes.c_longlong,
             "ddl_x6h_workspace": ctypes.c_longlong, "ddl_x6h_slots": ctypes.c_longlong, "ddl_bnf_fold_ws": ctypes.c_longlong, "ddl_bnf_fold_tickets": ctypes.c_longlong,
             "ddl_gram_f32_workspace": ctypes.c_longlong}

_OPTIONAL_SIGS: dict[str, list] = {}


def register_signatures(sigs: dict[str, list]) -> None:
    """Other op modules (llama kernels, ...) add their launchers here."""
    _OPTIONAL_SIGS.update(sigs)
    if _kernels is not None:
        _declare(_kernels, sigs)


def _declare(lib, sigs) -> None:
    for name, argt in sigs.items():
        fn = getattr(lib, name, None)
        if fn is None:
            continue
        fn.argtypes = argt
        fn.restype = _RESTYPES.get(name, ctypes.c_int)


def kernels_available() -> bool:
    return KERNEL_LIB_PATH.exists()


def kernels():
    """The loaded HIP kernel library (raises if it is missing: no silent fallback)."""
    global _kernels
    if _kernels is None:
        if not KERNEL_LIB_PATH.exists():
            raise RuntimeError(
                f"{KERNEL_LIB_PATH} is missing: build it with `python -m ddl25spring_amd._build` "
                "(hipcc --offload-arch=gfx950)")
        _ = torch.cuda.is_available()  # make sure torch's HIP runtime is the one we bind to
        lib = ctypes.CDLL(str(KERNEL_LIB_PATH), mode=ctypes.RTLD_GLOBAL)
        _declare(lib, _SIGS)
        _declare(lib, _OPTIONAL_SIGS)
        for name, size_fn, cls in (("ConvArgs", "ddl_conv_args_size", ConvArgs),
                                   ("BNArgs", "ddl_bn_args_size", BNArgs),
                                   ("BNBwdArgs", "ddl_bn_bwd_args_size", BNBwdArgs),
                                   ("HeadArgs", "ddl_head_args_size", HeadArgs),
                                   ("SGDArgs", "ddl_sgd_args_size", SGDArgs),
                                   ("SGDDirectArgs", "ddl_sgd_direct_args_size", SGDDirectArgs),
                                   ("AdamArgs", "ddl_adam_args_size", AdamArgs),
                                   ("ConvF32Args", "ddl_convf32_args_size", ConvF32Args),
                                   ("BNFArgs", "ddl_bnf_args_size", BNFArgs),
                                   ("BNFBwdArgs", "ddl_bnf_bwd_args_size", BNFBwdArgs),
                                   ("HeadFArgs", "ddl_headf_args_size", HeadFArgs)):
            f = getattr(lib, size_fn)
            f.restype = ctypes.c_int
            if f() != ctypes.sizeof(cls):
                raise RuntimeError(f"ABI mismatch for {name}: C {f()} vs ctypes {ctypes.sizeof(cls)}")
        _kernels = lib
    return _kernels


def runtime():
    """The host C++ runtime library (schedules / planners)."""
    global _runtime
    if _runtime is None:
        if not RUNTIME_LIB_PATH.exists():
            from .. import _build
            _build.build_runtime()
        lib = ctypes.CDLL(str(RUNTIME_LIB_PATH))
        p32 = ctypes.POINTER(ctypes.c_int32)
        lib.ddl_sched_build.argtypes = [i32, i32, i32, p32, i32]
        lib.ddl_sched_verify.argtypes = [p32, i32, i32]
        lib.ddl_plan_epoch.argtypes = [p32, i32, i32, i32, ctypes.POINTER(ctypes.c_uint64), i32, p32]
        lib.ddl_bucket_plan.argtypes = [ctypes.POINTER(ctypes.c_int64), i32, ctypes.c_int64, i32, p32]
        i64p, f64p = ctypes.POINTER(ctypes.c_int64), ctypes.POINTER(ctypes.c_double)
        lib.ddl_markov_walk.argtypes = [i64p, f64p, i32, i64p, f64p, i32, i32, ctypes.c_int64, i64p]
        for f in ("ddl_sched_build", "ddl_sched_verify", "ddl_plan_epoch", "ddl_bucket_plan",
                  "ddl_markov_walk"):
            getattr(lib, f).restype = ctypes.c_int
        _runtime = lib
    return _runtime


class KernelError(RuntimeError):
    pass


def check(rc: int, name: str) -> None:
    if rc != 0:
        raise KernelError(f"{name} failed with hipError {rc}")


def ptr(t) -> int | None:
    return None if t is None else t.data_ptr()


def stream() -> int:
    return torch.cuda.current_stream().cuda_stream


def loaded_library_paths() -> list[str]:
    """For diagnostics: which in-tree native libraries this process has mapped."""
    out = []
    try:
        with open(f"/proc/{os.getpid()}/maps") as f:
            for line in f:
                if str(LIBDIR) in line:
                    p = line.split()[-1]
                    if p not in out:
                        out.append(p)
    except OSError:
        pass
    return out
