"""C-ABI checks that run without a GPU: the library loads, exports every symbol
declared in include/ruserf_amd.h, and validates arguments before touching HIP."""
import ctypes as C

import numpy as np
import pytest

import ruserf_amd
from ruserf_amd import _lib


def test_library_loads_and_exports_every_declared_symbol():
    L = ruserf_amd.lib()
    syms = ruserf_amd.declared_symbols()
    assert len(syms) >= 15
    missing = [s for s in syms if not hasattr(L, s)]
    assert not missing, missing


def test_version_and_device_probe():
    L = ruserf_amd.lib()
    assert b"gfx950" in L.rsf_version()
    assert L.rsf_device_count() >= 0


def test_coord_defaults_match_coordinate_options_new():
    # CoordinateOptions::new (coordinate.rs:200-213)
    o = _lib.RsfCoordOpts()
    ruserf_amd.lib().rsf_coord_opts_default(C.byref(o))
    py = ruserf_amd.CoordinateOptions()
    for k in ["dimensionality", "vivaldi_error_max", "vivaldi_ce", "vivaldi_cc", "adjustment_window_size",
              "height_min", "latency_filter_size", "gravity_rho"]:
        assert getattr(o, k) == getattr(py, k)


def test_row_stride():
    L = ruserf_amd.lib()
    assert L.rsf_coord_row_stride(8) == 12  # 96-byte rows
    assert L.rsf_coord_row_stride(3) == 8
    assert L.rsf_coord_row_stride(16) == 20


def test_argument_validation_without_gpu():
    L = ruserf_amd.lib()
    h = C.c_void_p()
    o = ruserf_amd.CoordinateOptions().to_c()
    assert L.rsf_vivaldi_create(C.byref(h), 1, 0, 1, 4, C.byref(o), 1, 0) == _lib.RSF_ERR_ARG
    bad = ruserf_amd.CoordinateOptions(dimensionality=17).to_c()
    assert L.rsf_vivaldi_create(C.byref(h), 10, 0, 10, 4, C.byref(bad), 1, 0) == _lib.RSF_ERR_ARG
    assert b"dimensionality" in L.rsf_last_error()
    bad = ruserf_amd.CoordinateOptions(latency_filter_size=0).to_c()
    assert L.rsf_vivaldi_create(C.byref(h), 10, 0, 10, 4, C.byref(bad), 1, 0) == _lib.RSF_ERR_ARG


def test_coordinate_value_type():
    c = ruserf_amd.Coordinate.new()
    assert c.is_valid() and len(c.portion) == 8 and c.error == 1.5 and c.height == 10e-6
    c.portion[3] = float("nan")
    assert not c.is_valid()
    row = ruserf_amd.Coordinate.with_options(ruserf_amd.CoordinateOptions(dimensionality=3)).to_row()
    assert row.shape == (8,) and row[3] == 1.5 and row[5] == 10e-6
