"""ctypes binding of libhipdedisp.so (the C ABI in include/hipdedisp.h).

The shared library is built in-tree (pipeline2.0_amd/libhipdedisp.so) by
``__graft_entry__.build()`` / ``make -C pipeline2.0_amd/csrc``.  There is no
Python or CPU fallback: if the library is missing, importing the engine fails
loudly (HipDedispUnavailable) instead of silently computing elsewhere.
"""
import ctypes
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
# HD_LIB (A/B of two builds in one session): another build of the same library
LIB_PATH = os.environ.get("HD_LIB") or os.path.join(os.path.dirname(_HERE), "libhipdedisp.so")

HD_OK = 0
HD_E_INVAL = -1
HD_E_NODEV = -2
HD_E_HIP = -3
HD_E_NOMEM = -4
HD_E_STATE = -5
HD_E_IO = -6

HD_SUB_I16, HD_SUB_F32 = 0, 1
HD_DS_SUM, HD_DS_MEAN = 0, 1
HD_PAD_MEAN, HD_PAD_ZERO, HD_PAD_DM0 = 0, 1, 2
HD_ROUND_PRESTO, HD_ROUND_NEAREST = 0, 1
HD_PASS_SUB_INPUT = 1
HD_HOST_ONLY = -1
HD_EXT_SUBBANDS, HD_EXT_OFFSETS = 0, 1

ERROR_NAMES = {HD_E_INVAL: "HD_E_INVAL", HD_E_NODEV: "HD_E_NODEV", HD_E_HIP: "HD_E_HIP",
               HD_E_NOMEM: "HD_E_NOMEM", HD_E_STATE: "HD_E_STATE", HD_E_IO: "HD_E_IO"}

# Every symbol include/hipdedisp.h declares (checked by tests/test_abi.py).
EXPORTED = [
    "hd_version", "hd_opts_default", "hd_synth_default", "hd_device_count", "hd_open",
    "hd_close", "hd_last_error", "hd_sync", "hd_set_obs", "hd_set_chan_calib", "hd_set_mask",
    "hd_push_raw", "hd_synth_device", "hd_synth_host", "hd_plan_create", "hd_plan_destroy",
    "hd_plan_get_delays", "hd_plan_sub_params", "hd_run_subband", "hd_get_subbands",
    "hd_set_subbands", "hd_run_dedisp", "hd_plan_last_ms", "hd_plan_kernel", "hd_plan_set_variant",
    "hd_get_raw", "hd_plan_tables", "hd_run_subband_multi", "hd_push_raw_device", "hd_get_raw_device",
    "hd_push_raw_file", "hd_set_streams", "hd_touch_raw", "hd_stats_padvals", "hd_get_clean",
    "hd_get_subbands_window", "hd_get_series", "hd_write_series", "hd_wait_writes",
    "hd_set_slice", "hd_clip_stats", "hd_clip_set_stats", "hd_series_sum", "hd_series_sum_multi", "hd_series_fill", "hd_comm_unique_id", "hd_comm_init",
    "hd_comm_allreduce_sum_f64", "hd_slice_exchange_clip", "hd_comm_destroy",
    "hd_sp_widths", "hd_single_pulse", "hd_single_pulse_launch", "hd_single_pulse_collect", "hd_rfifind_stats",
    "hd_push_raw_file_band", "hd_fill_raw",
    "hd_realfft", "hd_fft_prepare", "hd_zap_ranges", "hd_zapbirds", "hd_rednoise_blocks", "hd_rednoise", "hd_get_fft",
    "hd_bary_diffbins", "hd_plan_set_bary", "hd_plan_data_end", "hd_run_dedisp_multi", "hd_plan_launch_passes", "hd_sp_prune",
    "hd_prefetch_raw_file", "hd_prefetch_raw_file_band", "hd_prefetch_fill", "hd_swap_raw",
    "hd_plan_extents", "hd_debug_fault",
]


class HipDedispUnavailable(RuntimeError):
    """libhipdedisp.so could not be loaded (not built, or no ROCm runtime)."""


class hd_obs(ctypes.Structure):
    _fields_ = [("nchan", ctypes.c_int32), ("nbits", ctypes.c_int32), ("npol", ctypes.c_int32),
                ("flip", ctypes.c_int32), ("dt", ctypes.c_double), ("lofreq", ctypes.c_double),
                ("df", ctypes.c_double), ("N", ctypes.c_int64), ("nsblk", ctypes.c_int32),
                ("_pad0", ctypes.c_int32), ("voverc", ctypes.c_double)]


class hd_opts(ctypes.Structure):
    _fields_ = [("sub_dtype", ctypes.c_int32), ("ds_mode", ctypes.c_int32),
                ("pad_mode", ctypes.c_int32), ("nibble_hi_first", ctypes.c_int32),
                ("be16", ctypes.c_int32), ("inf_roundtrip", ctypes.c_int32),
                ("clip_sigma", ctypes.c_float), ("sub_round", ctypes.c_int32)]


class hd_pass(ctypes.Structure):
    _fields_ = [("subdm", ctypes.c_double), ("lodm", ctypes.c_double), ("dmstep", ctypes.c_double),
                ("numdms", ctypes.c_int32), ("nsub", ctypes.c_int32), ("ds", ctypes.c_int32),
                ("flags", ctypes.c_int32), ("numout", ctypes.c_int64)]


class hd_extent(ctypes.Structure):
    _fields_ = [("kernel", ctypes.c_int32), ("region", ctypes.c_int32), ("ppc", ctypes.c_int32),
                ("_pad0", ctypes.c_int32), ("reach", ctypes.c_int64), ("size", ctypes.c_int64)]


_NPSR = 8


class hd_rows_src(ctypes.Structure):
    _fields_ = [("table_offset", ctypes.c_int64), ("row_bytes", ctypes.c_int64), ("col_offset", ctypes.c_int64),
                ("col_bytes", ctypes.c_int64), ("row0", ctypes.c_int64), ("nrows", ctypes.c_int64),
                ("block_bytes", ctypes.c_int64)]


class hd_synth(ctypes.Structure):
    _fields_ = [("seed", ctypes.c_uint64), ("base_level", ctypes.c_float),
                ("bandpass_slope", ctypes.c_float), ("noise_sigma", ctypes.c_float),
                ("npsr", ctypes.c_int32), ("nspulse", ctypes.c_int32),
                ("psr_period", ctypes.c_double * _NPSR), ("psr_dm", ctypes.c_double * _NPSR),
                ("psr_width", ctypes.c_double * _NPSR), ("psr_amp", ctypes.c_float * _NPSR),
                ("sp_time", ctypes.c_double * _NPSR), ("sp_dm", ctypes.c_double * _NPSR),
                ("sp_width", ctypes.c_double * _NPSR), ("sp_amp", ctypes.c_float * _NPSR),
                ("rfi_nchan", ctypes.c_int32), ("rfi_chan", ctypes.c_int32 * 8),
                ("rfi_amp", ctypes.c_float), ("burst_frac", ctypes.c_float),
                ("burst_len", ctypes.c_int32), ("burst_amp", ctypes.c_float),
                ("spike_frac", ctypes.c_float), ("spike_amp", ctypes.c_float)]


_lib = None


def load():
    """Load (once) and return the ctypes handle; raise HipDedispUnavailable if absent."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise HipDedispUnavailable(
            "%s is not built; run `python -c 'import __graft_entry__ as g; g.build()'` "
            "or `make -C pipeline2.0_amd/csrc`" % LIB_PATH)
    try:
        lib = ctypes.CDLL(LIB_PATH)
    except OSError as e:
        raise HipDedispUnavailable("cannot load %s: %s" % (LIB_PATH, e))
    P = ctypes.POINTER
    vp, i32, i64, f32p = ctypes.c_void_p, ctypes.c_int32, ctypes.c_int64, P(ctypes.c_float)
    sig = {
        "hd_version": (ctypes.c_char_p, []),
        "hd_opts_default": (None, [P(hd_opts)]),
        "hd_synth_default": (None, [P(hd_synth)]),
        "hd_device_count": (ctypes.c_int, [P(ctypes.c_int)]),
        "hd_open": (ctypes.c_int, [ctypes.c_int, P(vp)]),
        "hd_close": (ctypes.c_int, [vp]),
        "hd_last_error": (ctypes.c_char_p, [vp]),
        "hd_sync": (ctypes.c_int, [vp]),
        "hd_set_streams": (ctypes.c_int, [vp, i32]),
        "hd_touch_raw": (ctypes.c_int, [vp]),
        "hd_set_obs": (ctypes.c_int, [vp, P(hd_obs), P(hd_opts)]),
        "hd_set_chan_calib": (ctypes.c_int, [vp, f32p, f32p, f32p]),
        "hd_set_mask": (ctypes.c_int, [vp, P(ctypes.c_uint8), i32, i32, ctypes.c_double, P(ctypes.c_uint8), f32p]),
        "hd_stats_padvals": (ctypes.c_int, [f32p, i32, i32, f32p]),
        "hd_get_clean": (ctypes.c_int, [vp, f32p, P(ctypes.c_uint8), P(ctypes.c_uint8), P(i64)]),
        "hd_push_raw": (ctypes.c_int, [vp, vp, i64, i64]),
        "hd_synth_device": (ctypes.c_int, [vp, P(hd_synth)]),
        "hd_synth_host": (ctypes.c_int, [P(hd_obs), P(hd_synth), i64, i64, vp]),
        "hd_plan_create": (ctypes.c_int, [vp, P(hd_pass), P(vp)]),
        "hd_plan_destroy": (ctypes.c_int, [vp]),
        "hd_plan_get_delays": (ctypes.c_int, [vp, P(ctypes.c_int32), P(ctypes.c_int32)]),
        "hd_plan_sub_params": (ctypes.c_int, [vp, P(ctypes.c_double), P(ctypes.c_double),
                                              P(ctypes.c_double), P(ctypes.c_int64)]),
        "hd_run_subband": (ctypes.c_int, [vp]),
        "hd_get_subbands": (ctypes.c_int, [vp, vp]),
        "hd_get_subbands_window": (ctypes.c_int, [vp, i64, i64, vp]),
        "hd_get_series": (ctypes.c_int, [vp, i32, i32, i64, i64, f32p]),
        "hd_write_series": (ctypes.c_int, [vp, P(ctypes.c_char_p), i32]),
        "hd_wait_writes": (ctypes.c_int, [vp, P(ctypes.c_double), P(i64)]),
        "hd_set_subbands": (ctypes.c_int, [vp, vp]),
        "hd_run_dedisp": (ctypes.c_int, [vp, f32p]),
        "hd_run_dedisp_multi": (ctypes.c_int, [P(vp), i32]),
        "hd_sp_prune": (ctypes.c_int, [vp, i64, i32, P(i32), i32, i64, i64, P(i64)]),
        "hd_plan_launch_passes": (ctypes.c_int, [vp, P(i32)]),
        "hd_plan_last_ms": (ctypes.c_int, [vp, f32p, f32p]),
        "hd_plan_kernel": (ctypes.c_int, [vp, ctypes.c_char_p, ctypes.c_int32]),
        "hd_plan_set_variant": (ctypes.c_int, [vp, i32]),
        "hd_get_raw": (ctypes.c_int, [vp, vp, i64, i64]),
        "hd_run_subband_multi": (ctypes.c_int, [P(vp), i32]),
        "hd_push_raw_device": (ctypes.c_int, [vp, vp, i64, i64]),
        "hd_get_raw_device": (ctypes.c_int, [vp, vp, i64, i64]),
        "hd_push_raw_file": (ctypes.c_int, [vp, ctypes.c_char_p, P(hd_rows_src), i64, P(ctypes.c_double),
                                            P(ctypes.c_double)]),
        "hd_push_raw_file_band": (ctypes.c_int, [vp, ctypes.c_char_p, P(hd_rows_src), i64, i64, i64, i64, i64,
                                                 P(ctypes.c_double), P(ctypes.c_double)]),
        "hd_fill_raw": (ctypes.c_int, [vp, i64, i64, i32]),
        "hd_set_slice": (ctypes.c_int, [vp, i64, i64]),
        "hd_clip_stats": (ctypes.c_int, [vp, i64, vp]),
        "hd_clip_set_stats": (ctypes.c_int, [vp, vp]),
        "hd_series_sum": (ctypes.c_int, [vp, i32, i64, i64, P(ctypes.c_double)]),
        "hd_series_sum_multi": (ctypes.c_int, [P(vp), i32, i32, P(i64), P(i64), P(ctypes.c_double)]),
        "hd_comm_unique_id": (ctypes.c_int, [P(ctypes.c_uint8)]),
        "hd_comm_init": (ctypes.c_int, [vp, P(ctypes.c_uint8), i32, i32]),
        "hd_comm_allreduce_sum_f64": (ctypes.c_int, [vp, vp, i64]),
        "hd_slice_exchange_clip": (ctypes.c_int, [vp, i64, i64]),
        "hd_comm_destroy": (ctypes.c_int, [vp]),
        "hd_series_fill": (ctypes.c_int, [vp, i64, ctypes.c_float]),
        "hd_rfifind_stats": (ctypes.c_int, [vp, i32, f32p, f32p, f32p]),
        "hd_realfft": (ctypes.c_int, [vp]),
        "hd_fft_prepare": (ctypes.c_int, [vp]),
        "hd_zap_ranges": (ctypes.c_int, [P(ctypes.c_double), P(ctypes.c_double), i32, i64, P(ctypes.c_int32), i32,
                                         P(ctypes.c_int32)]),
        "hd_zapbirds": (ctypes.c_int, [vp, P(ctypes.c_double), P(ctypes.c_double), i32]),
        "hd_rednoise_blocks": (ctypes.c_int, [i64, ctypes.c_double, i32, i32, ctypes.c_double, P(ctypes.c_int32), i32,
                                              P(ctypes.c_int32)]),
        "hd_rednoise": (ctypes.c_int, [vp, i32, i32, ctypes.c_double, ctypes.c_double]),
        "hd_get_fft": (ctypes.c_int, [vp, i32, i32, f32p]),
        "hd_bary_diffbins": (ctypes.c_int, [P(ctypes.c_double), P(ctypes.c_double), i32, ctypes.c_double,
                                            ctypes.c_double, P(ctypes.c_int32), i32, P(ctypes.c_int32)]),
        "hd_plan_set_bary": (ctypes.c_int, [vp, P(ctypes.c_int32), i32]),
        "hd_plan_data_end": (ctypes.c_int, [vp, P(ctypes.c_int64)]),
        "hd_prefetch_raw_file": (ctypes.c_int, [vp, ctypes.c_char_p, P(hd_rows_src), i64]),
        "hd_prefetch_raw_file_band": (ctypes.c_int, [vp, ctypes.c_char_p, P(hd_rows_src), i64, i64, i64, i64, i64]),
        "hd_prefetch_fill": (ctypes.c_int, [vp, i64, i64, i32]),
        "hd_swap_raw": (ctypes.c_int, [vp, P(ctypes.c_double), P(ctypes.c_double)]),
        "hd_sp_widths": (ctypes.c_int, [ctypes.c_double, ctypes.c_double, P(ctypes.c_int32), P(ctypes.c_int32)]),
        "hd_single_pulse": (ctypes.c_int, [vp, ctypes.c_double, ctypes.c_double, ctypes.c_double, vp, i64, P(i64),
                                           P(ctypes.c_uint8), P(i64)]),
        "hd_single_pulse_launch": (ctypes.c_int, [vp, ctypes.c_double, ctypes.c_double, ctypes.c_double]),
        "hd_single_pulse_collect": (ctypes.c_int, [vp, vp, i64, P(i64), P(ctypes.c_uint8), P(i64)]),
        "hd_plan_extents": (ctypes.c_int, [P(hd_obs), P(hd_opts), P(hd_pass), P(hd_extent), i32, P(i32)]),
        "hd_debug_fault": (ctypes.c_int, [vp]),
        "hd_plan_tables": (ctypes.c_int, [P(hd_obs), P(hd_opts), P(hd_pass), P(ctypes.c_int32),
                                          P(ctypes.c_int32), P(ctypes.c_double), P(ctypes.c_double),
                                          P(ctypes.c_double)]),
    }
    for name, (res, args) in sig.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    _lib = lib
    return lib


def last_error(ctx=None):
    msg = load().hd_last_error(ctx)
    return msg.decode() if msg else ""
