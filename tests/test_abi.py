"""CPU: the C-ABI library loads and exports every symbol include/wv_knn.h
declares (no compute calls -- there is no GPU here)."""
import os
import re

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def header_functions():
    src = open(os.path.join(REPO, "include", "wv_knn.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    names = re.findall(r"\b(wv_[a-z0-9_]+)\s*\(", src)
    return sorted(set(names))


def test_header_declares_entry_points():
    names = header_functions()
    for must in ["wv_index_create", "wv_index_add_batch", "wv_index_search_by_vector_batch",
                 "wv_index_search_by_vector_distance", "wv_distance_batch", "wv_last_error"]:
        assert must in names


def test_library_exports_every_header_symbol(wv):
    lib = wv.load()
    missing = [n for n in header_functions() if not hasattr(lib, n)]
    assert not missing, missing


def test_ctypes_signatures_cover_header(wv):
    from weaviate_amd import _lib
    assert set(header_functions()) == set(_lib.SIGNATURES)


def test_no_fallback_when_library_missing(monkeypatch, tmp_path):
    from weaviate_amd import _lib
    monkeypatch.setattr(_lib, "_lib", None)
    monkeypatch.setattr(_lib, "LIB_PATH", str(tmp_path / "missing.so"))
    import pytest
    with pytest.raises(RuntimeError, match="no CPU fallback"):
        _lib.load()


def test_variant_rule_matches_reference_dispatch(wv):
    """distancer/l2_amd64.go:19-26: AVX-512 kernels only with AMX-BF16 && AVX512."""
    lib = wv.load()
    flags = open("/proc/cpuinfo").read().split()
    expect = 2 if ("amx_bf16" in flags and "avx512f" in flags) else 1
    assert lib.wv_resolve_variant(0) == expect
    assert lib.wv_resolve_variant(1) == 1 and lib.wv_resolve_variant(2) == 2


def test_validate_user_config_update_host_only(wv):
    """flat.ValidateUserConfigUpdate (flat/index.go:1106-1154): host logic, no GPU."""
    import pytest
    from weaviate_amd.flat import validate_user_config_update as v
    base = dict(distance="cosine", bq=True, rescore_limit=10)
    v(base, dict(base, rescore_limit=300))  # rescore is mutable
    with pytest.raises(wv.WeaviateError, match='distance is immutable: attempted change from "cosine" to "l2-squared"'):
        v(base, dict(base, distance="l2-squared"))
    with pytest.raises(wv.WeaviateError, match='bq is immutable: attempted change from "true" to "false"'):
        v(base, dict(base, bq=False))
    with pytest.raises(wv.WeaviateError, match='pq is immutable: attempted change from "false" to "true"'):
        v(dict(distance="dot"), dict(distance="dot", pq={"segments": 4}))
    with pytest.raises(wv.WeaviateError, match='rq is immutable: attempted change from "false" to "true"'):
        v(dict(distance="dot"), dict(distance="dot", rq={"bits": 8}))
    with pytest.raises(wv.WeaviateError, match='rq.bits is immutable: attempted change from "8" to "1"'):
        v(dict(distance="dot", rq={"bits": 8}), dict(distance="dot", rq={"bits": 1}))


def test_multi_config_validation_without_gpu():
    """wv_multi_create refuses inconsistent worlds before touching a device:
    the host language gets the error text, no GPU needed."""
    import ctypes as C
    from weaviate_amd import _lib
    from weaviate_amd.flat import make_config
    lib = _lib.load()
    devs = (C.c_int32 * 2)(0, 0)

    def create(world, rank0, n_local, transport, stride=100, uid=None, cfg=None):
        mc = _lib.WvMultiConfig(cfg or make_config(distance="cosine", dims=8), world, rank0, n_local,
                                C.cast(devs, C.POINTER(C.c_int32)), stride, transport, uid, None, None, None)
        h = C.c_void_p()
        rc = lib.wv_multi_create(C.byref(mc), C.byref(h))
        return rc, (lib.wv_last_error() or b"").decode()

    assert create(2, 0, 1, 0) == (_lib.WV_ERR_INVALID, "local transport: every rank must be a local shard")
    rc, msg = create(2, 1, 1, 1)
    assert rc == _lib.WV_ERR_INVALID and "unique id" in msg
    rc, msg = create(2, 0, 1, 2)
    assert rc == _lib.WV_ERR_INVALID and "callbacks" in msg
    rc, msg = create(2, 2, 1, 0)
    assert rc == _lib.WV_ERR_INVALID and "invalid multi config" in msg
    rc, msg = create(2, 0, 2, 0, stride=0)
    assert rc == _lib.WV_ERR_INVALID and "id_stride" in msg
    bad = make_config(distance="cosine", dims=8, bq=True)
    bad.compression = 9  # every WV_COMPRESSION_* is taken (BQ, PQ, rq-8 / rq-1, SQ); others are refused
    rc, msg = create(1, 0, 1, 0, cfg=bad)
    assert rc == _lib.WV_ERR_INVALID and "unknown compression" in msg
    rc, msg = create(1, 0, 1, 7)
    assert rc == _lib.WV_ERR_INVALID and "unknown transport" in msg
