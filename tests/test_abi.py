"""The C-ABI library loads on the CPU host and exports exactly what include/*.h declares."""

import ctypes
import glob
import os
import re

import pytest

from plato_amd import _lib

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared_symbols(pattern="plato_agg.h"):
    names = set()
    for header in glob.glob(os.path.join(ROOT, "include", pattern)):
        text = open(header).read()
        text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
        names.update(re.findall(r"\b(plato_(?:agg|ingest)_\w+)\s*\(", text))
    return names


def test_headers_declare_the_boundary():
    names = declared_symbols()
    for required in ("plato_agg_fedavg_weights", "plato_agg_fedavg_deltas", "plato_agg_compute_deltas",
                     "plato_agg_update_weights", "plato_agg_cast_f32_i64", "plato_agg_mix_weights",
                     "plato_agg_last_error", "plato_agg_abi_version"):
        assert required in names


def test_library_exports_every_declared_symbol():
    if not os.path.exists(_lib.LIB_PATH):
        pytest.skip("library not built (run __graft_entry__.build())")
    handle = ctypes.CDLL(_lib.LIB_PATH)
    for name in declared_symbols():
        assert hasattr(handle, name), name
    # and the Python binding knows the signature of each
    assert declared_symbols() == set(_lib.SIGNATURES)
    # the tuning entry points are not part of the product library
    for name in declared_symbols("plato_agg_tune.h"):
        assert not hasattr(handle, name), name


def test_tuning_library_exports_both_headers():
    if not os.path.exists(_lib.TUNE_LIB_PATH):
        pytest.skip("tuning library not built (run __graft_entry__.build())")
    handle = ctypes.CDLL(_lib.TUNE_LIB_PATH)
    tune = declared_symbols("plato_agg_tune.h")
    assert tune == set(_lib.TUNE_SIGNATURES)
    for name in declared_symbols() | tune:
        assert hasattr(handle, name), name


def test_ingest_library_exports_its_header():
    from plato_amd import ingest

    if not os.path.exists(ingest.LIB_PATH):
        pytest.skip("ingest library not built")
    handle = ctypes.CDLL(ingest.LIB_PATH)
    names = declared_symbols("plato_ingest.h")
    assert names == {"plato_ingest_last_error", "plato_ingest_parse", "plato_ingest_gather", "plato_ingest_join",
                     "plato_ingest_read_fd", "plato_ingest_pack",
                     "plato_ingest_zstd_available", "plato_ingest_zstd_content_size",
                     "plato_ingest_zstd_decompress", "plato_ingest_zstd_bound", "plato_ingest_zstd_compress"}
    for name in names:
        assert hasattr(handle, name), name


def test_binding_loads_and_reports_abi():
    if not os.path.exists(_lib.LIB_PATH):
        pytest.skip("library not built")
    lib = _lib.lib()
    assert lib.plato_agg_abi_version() == _lib.ABI_VERSION
    assert _lib.tune().plato_agg_tune_num_variants() >= 1


def test_argument_errors_are_raised_without_gpu_work():
    """Invalid arguments are rejected on the host (no launch), mapped to ValueError."""
    if not os.path.exists(_lib.LIB_PATH):
        pytest.skip("library not built")
    with pytest.raises(ValueError, match="K must be"):
        _lib.call("plato_agg_fedavg_weights", None, None, None, None, 0, None, None, None, None, 16, 0, None)
    with pytest.raises(ValueError, match="null"):
        _lib.call("plato_agg_fedavg_weights", None, None, 8, None, 2, None, None, None, None, 16, 0, None)
    with pytest.raises(ValueError, match="aligned"):
        _lib.call("plato_agg_fedavg_weights", 8, None, 8, None, 2, 4, None, 4, None, 16, 0, None)
    with pytest.raises(ValueError, match="modulus"):
        _lib.call("plato_agg_fill_synth_i64", 8, None, 4, 0, 0, 0, None)
    # FedAdp's boundary table is addressed with 32-bit byte offsets of 1 KiB rows: a segment count whose
    # table would reach 2^22 rows is refused, not wrapped
    a = 1 << 12  # any 256-byte-aligned non-null address: nothing is dereferenced on this path
    with pytest.raises(ValueError, match="boundary table"):
        _lib.call("plato_agg_fedadp_dots", a, a, a, 1, a, None, a, (1 << 21) - 1, 1 << 20, 1 << 20, 0, 0.01, 1,
                  a, a, a, None)
    with pytest.raises(ValueError, match="flags"):  # only PLATO_AGG_FEDADP_TABLES_READY is defined
        _lib.call("plato_agg_fedadp_dots_ex", a, a, a, 1, a, None, a, 1, 64, 64, 0, 0.01, 1, a, a, a, None, 2)
    from plato_amd.engine import AggregationRound

    assert AggregationRound.fedadp_boundary_rows((1 << 21) - 1, 0) >= AggregationRound.FEDADP_MAX_BND


def test_engine_refuses_without_gpu():
    import torch

    if torch.cuda.is_available():
        pytest.skip("GPU present")
    from plato_amd.engine import FedAvgEngine

    with pytest.raises(RuntimeError, match="no ROCm GPU"):
        FedAvgEngine()
