"""The C-ABI library loads and exports exactly what include/pnr.h declares
(no compute calls: CPU-only)."""
import os
import re
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HDR = os.path.join(ROOT, "include", "pnr.h")
LIB = os.path.join(ROOT, "pointnerf_amd", "libpnr.so")


def header_functions():
    src = open(HDR).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(pnr_[a-z0-9_]+)\s*\(", src)))


@pytest.fixture(scope="module")
def built():
    if not os.path.exists(LIB):
        subprocess.check_call(["make", "-C", ROOT, "-j8", "pointnerf_amd/libpnr.so"])
    return LIB


def test_header_declares_the_boundary():
    fns = header_functions()
    for must in ("pnr_create", "pnr_destroy", "pnr_grid_build", "pnr_query", "pnr_query_compact",
                 "pnr_aggregate_fwd", "pnr_composite_fwd", "pnr_ray_march_fwd", "pnr_grid_stats_get"):
        assert must in fns


def test_library_exports_every_header_symbol(built):
    out = subprocess.check_output(["nm", "-D", "--defined-only", built], text=True)
    exported = set(re.findall(r" T (pnr_[a-z0-9_]+)", out))
    missing = set(header_functions()) - exported
    assert not missing, missing
    extra = exported - set(header_functions())     # no debug / ablation entry points in the product
    assert not extra, extra


def test_ctypes_binding_covers_header_and_loads(built):
    from pointnerf_amd import _lib as L
    assert set(L.SIGNATURES) == set(header_functions())
    lib = L.lib()
    assert lib.pnr_abi_version() == L.ABI_VERSION
    # argument validation runs on the host and never throws across the ABI
    assert lib.pnr_create(0, None) == L.PNR_EINVAL
    assert b"null" in lib.pnr_last_error()
    assert lib.pnr_grid_build(None, None, 0, None, None) == L.PNR_EINVAL
    assert lib.pnr_query(None, None, None, None, None) == L.PNR_EINVAL
    assert lib.pnr_aggregate_fwd(None, None, None, None, None, None, None, 0, None) == L.PNR_EINVAL
    assert lib.pnr_destroy(None) == L.PNR_OK


def test_scan_refuses_an_output_without_room_for_the_total(built):
    """exclusive_scan stores the grand total at out[n]: an `out` of n entries is
    refused on the host before any launch (the r05 used_map overrun).
    The pointers are never dereferenced: the check runs first."""
    from pointnerf_amd import _lib as L
    lib = L.lib()
    fake = L.c_void_p(0x1000)
    n = 1000
    nb = L.c_size_t(0)
    assert lib.pnr_scan_scratch_bytes(n, L.ctypes.byref(nb)) == L.PNR_OK
    rc = lib.pnr_exclusive_scan_i32(fake, n, None, fake, n, None, fake, nb.value, None)
    assert rc == L.PNR_EINVAL
    assert b"out holds 1000 entries" in lib.pnr_last_error()


def test_code_object_targets_gfx950(built):
    data = open(built, "rb").read()
    assert b"amdgcn-amd-amdhsa--gfx950" in data
    for other in (b"--gfx90a", b"--gfx942", b"--gfx1100"):
        assert other not in data
