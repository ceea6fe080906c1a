"""ctypes signatures of ``libdw_kernels.so`` (one place, checked at load)."""

import ctypes as c

vp, i64, i32, u32, u64, f32, cp = (c.c_void_p, c.c_int64, c.c_int, c.c_uint32, c.c_uint64,
                                   c.c_float, c.c_char_p)

SIGS = {
    # fp8.hip
    "dw_fp8_cast_amax": (i32, [vp, i32, vp, vp, vp, i64, i32, vp]),
    "dw_fp8_update_scales": (i32, [vp, vp, vp, vp, vp, i32, i32, i32, f32, vp]),
    "dw_fp8_cast_t": (i32, [vp, i32, vp, vp, vp, vp, i32, i32, i32, vp]),
    # ckpt_copy.hip
    "dw_multi_copy": (i32, [vp, i64, vp]),
    "dw_gemm_dgelu": (i32, [vp, vp, vp, vp, i32, i32, i32, vp]),
    "dw_gemm_dgelu_bgrad": (i32, [vp, vp, vp, vp, vp, i32, i32, i32, vp]),
    "dw_gemm_wgrad_bgradb": (i32, [vp, vp, vp, vp, i32, i32, i32, i32, vp]),
    "dw_multi_copy_grid": (i32, [vp, i64, i32, vp]),
    "dw_multi_copy_variant": (i32, [vp, i64, i32, i32, vp]),
    "dw_fill_u32": (i32, [vp, i64, u32, vp]),
    "dw_host_register": (i32, [vp, u64]),
    "dw_host_unregister": (i32, [vp]),
    "dw_host_registered": (i32, [vp]),
    "dw_memcpy_async": (i32, [vp, vp, u64, i32, vp]),
    "dw_stream_sync": (i32, [vp]),
    "dw_event_sync": (i32, [vp]),
    "dw_stream_create_cumask": (vp, [i32, c.POINTER(i32)]),
    "dw_stream_destroy": (i32, [vp]),
    "dw_stream_create_prio": (vp, [i32, c.POINTER(i32)]),
    "dw_host_device_ptr": (vp, [vp]),
    "dw_stream_copy": (i32, [vp, vp, u64, i32, vp]),
    "dw_device_malloc": (i32, [u64, c.POINTER(vp)]),
    "dw_device_free": (i32, [vp]),
    "dw_ipc_handle_size": (i32, []),
    "dw_ipc_get_handle": (i32, [vp, vp]),
    "dw_ipc_open_handle": (i32, [vp, c.POINTER(vp)]),
    "dw_ipc_close_handle": (i32, [vp]),
    "dw_mem_get_info": (i32, [c.POINTER(u64), c.POINTER(u64)]),
    "dw_hip_error_string": (cp, [i32]),
    "dw_kernels_abi_version": (i32, []),
    "dw_preload_code_objects": (i32, []),  # preload.hip
    # xpu_timer.hip
    "dw_xt_start": (i32, [c.c_double, i32]),
    "dw_xt_stop": (i32, []),
    "dw_xt_flush": (i32, [c.c_double]),
    "dw_xt_key": (i32, [cp]),
    "dw_xt_begin": (i64, [i32, vp]),
    "dw_xt_end": (i32, [i64, c.c_double, vp]),
    "dw_xt_snapshot": (i32, [c.c_char_p, i32]),
    "dw_xt_hang": (i32, [c.c_char_p, i32, c.POINTER(c.c_double)]),
    "dw_xt_reset": (None, []),
    "dw_xt_pending": (i64, []),
    # quant.hip
    "dw_quantize": (i32, [vp, i32, vp, vp, i64, i64, i32, i32, vp]),
    "dw_dequant_reduce": (i32, [vp, vp, vp, i32, i32, i64, i64, i32, i32, vp]),
    # optim.hip
    "dw_adam_flat": (i32, [vp, i32, vp, vp, i32, vp, vp, vp, i64, i64, f32, f32, f32, f32, f32,
                           f32, f32, i32, vp, vp]),
    "dw_adam_replay": (i32, [vp, i32, vp, vp, vp, i64, i32, vp, i32, vp, vp, vp, vp, f32, f32, f32, f32, i32, vp,
                             i32, vp]),
    "dw_agd_flat": (i32, [vp, i32, vp, vp, i32, vp, vp, vp, i64, i64, f32, f32, f32, f32, f32,
                          f32, f32, f32, f32, vp, vp]),
    "dw_sumsq_flat": (i32, [vp, i32, i64, vp, vp, vp]),
    "dw_clip_coef": (i32, [vp, f32, f32, vp, vp, vp]),
    "dw_scale_flat": (i32, [vp, i32, i64, vp, vp]),
    # optim_multi.hip
    "dw_mt_adam": (i32, [vp, vp, i64, vp, vp, i32, vp]),
    "dw_mt_adam_grid": (i32, [vp, vp, i64, vp, vp, i32, i32, vp]),
    "dw_mt_sumsq": (i32, [vp, vp, i64, vp, vp, vp]),
    "dw_mt_hyper_size": (i32, []),
    "dw_mt_chunk": (i32, []),
    # norm.hip
    "dw_norm_fwd": (i32, [vp, vp, vp, vp, vp, vp, i64, i32, f32, i32, vp]),
    "dw_norm_bwd_blocks": (i32, [i64]),
    "dw_norm_bwd": (i32, [vp, vp, vp, vp, vp, vp, vp, vp, vp, i64, i32, i32, i32, vp]),
    # elementwise.hip
    "dw_bias_gelu_fwd": (i32, [vp, vp, vp, vp, i64, i32, vp]),
    "dw_gelu_bwd": (i32, [vp, vp, vp, i64, vp]),
    "dw_colsum_parts": (i32, [i64]),
    "dw_colsum": (i32, [vp, i64, i32, vp, vp, i32, vp]),
    # optim_lowbit.hip
    "dw_qadamw": (i32, [vp, vp, vp, vp, vp, vp, i64, i64, i32, i32, i32, f32, f32, f32, f32, f32, f32, f32, f32,
                        vp]),
    # colred.hip
    "dw_colsum_acc": (i32, [vp, i64, i32, vp, vp, i32, i32, vp, vp]),
    "dw_gelu_bwd_dbias": (i32, [vp, vp, vp, i64, i32, vp, vp, i32, i32, vp, vp]),
    "dw_norm_bwd2": (i32, [vp, vp, vp, vp, vp, vp, vp, vp, vp, vp, i64, i32, i32, i32, i32, vp, vp]),
    "dw_norm_bwd3": (i32, [vp, vp, vp, vp, vp, vp, vp, vp, vp, vp, vp, i64, i64, i32, i32, i32, i32, vp, vp, vp, vp]),
    "dw_colred_det_floats": (i64, [i64, i32, i32]),
    "dw_add_norm_fwd": (i32, [vp, vp, vp, vp, vp, vp, vp, vp, i64, i32, f32, i32, vp]),
    "dw_swiglu_fwd": (i32, [vp, vp, i64, i32, vp]),
    "dw_swiglu_bwd": (i32, [vp, vp, vp, i64, i32, vp]),
    "dw_rope": (i32, [vp, vp, vp, vp, i64, i32, i32, i32, i32, vp, i32, vp]),
    "dw_qkv_rope": (i32, [vp, vp, vp, vp, vp, vp, i64, i32, i32, i32, i32, i32, vp, i32, vp]),
    # grouped_gemm.hip
    "dw_grouped_gemm": (i32, [i32, vp, vp, vp, vp, i32, i32, i32, i32, i32, c.c_longlong, c.c_longlong,
                              c.c_longlong, c.c_longlong, c.c_longlong, vp]),
    # xent.hip
    "dw_xent_fwd": (i32, [vp, vp, vp, vp, vp, vp, i64, i32, i64, i64, f32, vp]),
    "dw_xent_bwd": (i32, [vp, vp, vp, vp, i32, vp, i64, i32, i64, i64, f32, vp]),
}

OPTIONAL = {
    # attention kernels (attn_fwd.hip / attn_bwd.hip)
    "dw_attn_fwd": (i32, [vp, vp, vp, vp, vp, i32, i32, i32, i32, i32, i32, f32, i32, vp]),
    "dw_attn_bwd": (i32, [vp, vp, vp, vp, vp, vp, vp, vp, vp, vp, vp, i32, i32, i32, i32, i32,
                          i32, f32, i32, vp]),
    "dw_attn_bwd_workspace": (i64, [i32, i32, i32, i32]),
    "dw_attn_fwd_strided": (i32, [vp, vp, vp, vp, vp, i32, i32, i32, i32, i32, vp, i32, f32, i32, vp]),
    "dw_attn_bwd_strided": (i32, [vp, vp, vp, vp, vp, vp, vp, vp, vp, vp, i32, i32, i32, i32, i32, vp, i32, f32,
                                  i32, vp]),
    "dw_attn_decode": (i32, [vp, vp, vp, vp, vp, vp, vp, i32, i32, i32, i32, i32, i32, vp, f32, vp]),
    "dw_attn_fwd_varlen": (i32, [vp, vp, vp, vp, vp, vp, vp, i32, i32, i32, i32, i32, i32, vp, i32, f32, vp]),
    "dw_attn_bwd_varlen": (i32, [vp, vp, vp, vp, vp, vp, vp, vp, vp, vp, vp, vp, i32, i32, i32, i32, i32, i32, i32,
                                 i32, vp, i32, f32, vp]),
    # extended masks (window / GLM prefix / bias / ALiBi / dropout): last vp = AttnExtArgs*
    "dw_attn_fwd_ext": (i32, [vp, vp, vp, vp, vp, i32, i32, i32, i32, i32, vp, i32, f32, vp, vp]),
    "dw_attn_bwd_ext": (i32, [vp, vp, vp, vp, vp, vp, vp, vp, vp, vp, i32, i32, i32, i32, i32, vp, i32, f32, vp, vp]),
    "dw_attn_fwd_varlen_ext": (i32, [vp, vp, vp, vp, vp, vp, vp, i32, i32, i32, i32, i32, i32, i32, vp, i32, f32, vp,
                                     vp]),
    "dw_attn_bwd_varlen_ext": (i32, [vp, vp, vp, vp, vp, vp, vp, vp, vp, vp, vp, vp, i32, i32, i32, i32, i32, i32,
                                     i32, i32, vp, i32, f32, vp, vp]),
    "dw_attn_dropout_mask": (i32, [vp, i32, i32, i32, f32, u64, u64, vp]),
    # moe_permute.hip
    "dw_moe_regroup": (i32, [vp, vp, vp, i32, i32, i64, i32, i32, vp]),
}


def declare(lib):
    for name, (res, args) in SIGS.items():
        f = getattr(lib, name)
        f.restype = res
        f.argtypes = args
    for name, (res, args) in OPTIONAL.items():
        f = getattr(lib, name, None)
        if f is not None:
            f.restype = res
            f.argtypes = args
