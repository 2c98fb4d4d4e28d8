"""CPU-side checks of the drop-in boundary: libacnerf.so loads (no GPU needed for dlopen) and
exports every entry point declared in include/acnerf.h; the Python binding declares exactly that
set; no compute call is made here."""
import ctypes
import re
from pathlib import Path

REPO = Path(__file__).resolve().parent.parent


def declared_symbols():
    text = (REPO / "include" / "acnerf.h").read_text()
    return sorted(set(re.findall(r"^(?:int|size_t)\s+(acn_\w+)\s*\(", text, re.M)))


def test_header_declares_expected_entry_points():
    syms = declared_symbols()
    for s in ["acn_version", "acn_last_error", "acn_hashgrid_fwd", "acn_hashgrid_bwd", "acn_sh_fwd",
              "acn_workspace_bytes", "acn_field_fwd", "acn_volume_render_fwd", "acn_render_stratified_fwd",
              "acn_get_rays"]:
        assert s in syms, s


def test_library_loads_and_exports_every_declared_symbol():
    import torch  # noqa: F401  (binds torch's HIP runtime first, as the package does)
    from adaptive_city_nerf_amd import _lib
    L = _lib.lib()
    for s in declared_symbols():
        assert hasattr(L, s), f"libacnerf.so does not export {s}"
    assert L.acn_version() == 1
    assert set(_lib.exported_symbols()) == set(declared_symbols())
    assert L.acn_workspace_bytes(1) > 50_000 and L.acn_workspace_bytes(4) == 4 * L.acn_workspace_bytes(1)
    # the scratch of acn_render_stratified_fwd_ordered: the ray order (n <= 8192 rays, 4 B each)
    order = lambda n: 4 * n if n <= 8192 else 0  # noqa: E731
    assert [L.acn_render_order_bytes(n) for n in (0, 1, 4096, 8192, 8193)] == [0] + [order(n) for n in (1, 4096, 8192,
                                                                                                         8193)]


def test_argument_errors_are_reported_without_a_gpu():
    """Shape/argument validation happens before any HIP call, so it is testable on CPU."""
    from adaptive_city_nerf_amd import _lib
    L = _lib.lib()
    res = (ctypes.c_int32 * 40)()
    st = L.acn_hashgrid_fwd(None, 10, None, res, 40, 20, 2, 1, None, None)
    assert st == -1
    buf = ctypes.create_string_buffer(256)
    L.acn_last_error(buf, 256)
    assert b"levels" in buf.value
    assert L.acn_sh_fwd(None, 4, 7, None, None) == -1
    assert L.acn_render_stratified_fwd(None, 4, 1, None, None, None, -1, None, 1.0, 0.0, None, 0, None, None,
                                       None, None, None) == -1
    assert L.acn_render_stratified_fwd_ordered(None, 4, 1, None, None, None, -1, None, 1.0, 0.0, None, 0, None,
                                               None, None, None, None, 0, None) == -1
