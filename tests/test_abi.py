"""The C-ABI library builds, loads without a GPU and exports every declared symbol."""
import os
import re

from conftest import REPO


def declared_symbols():
    hdr = open(os.path.join(REPO, "include", "gcolor.h")).read()
    hdr = re.sub(r"/\*.*?\*/", "", hdr, flags=re.S)
    return sorted(set(re.findall(r"\b(gc_[a-z_]+)\s*\(", hdr)))


def test_header_matches_binding_list():
    from gcolor_amd import _native
    assert declared_symbols() == sorted(_native.EXPORTS)


def test_library_exports_every_declared_symbol():
    from gcolor_amd import _native
    lib = _native.load()
    for name in declared_symbols():
        assert getattr(lib, name) is not None, name


def test_gen_uniform_host_entry_point():
    """gc_gen_uniform is host code: callable without a GPU."""
    import numpy as np
    from gcolor_amd.engine import uniform_csr
    rp, col = uniform_csr(5000, 8, seed=3)
    deg = np.diff(rp)
    assert deg.max() <= 8
    # simple and symmetric
    n = 5000
    src = np.repeat(np.arange(n), deg)
    assert not np.any(src == col)
    a = np.sort(src * n + col)
    b = np.sort(col.astype(np.int64) * n + src)
    assert np.array_equal(a, b) and np.unique(a).shape == a.shape
    rp2, col2 = uniform_csr(5000, 8, seed=3)
    assert np.array_equal(rp, rp2) and np.array_equal(col, col2)


def test_last_error_is_callable():
    from gcolor_amd import _native
    assert isinstance(_native.load().gc_last_error(), bytes)


def test_input_stream_is_set_around_one_call_and_restored():
    """engine._input_stream names the caller's stream for one call (gc_set_input_stream) and
    restores the device-wide ordering afterwards, also when the call raises; None leaves the
    library untouched (no GPU needed: the library's setter only records the value)."""
    import ctypes
    from gcolor_amd import engine

    calls = []

    class Lib:
        def gc_set_input_stream(self, stream, enable):
            calls.append((stream.value if isinstance(stream, ctypes.c_void_p) else stream, enable))
            return 0

    lib = Lib()
    with engine._input_stream(lib, None):
        pass
    assert calls == []
    with engine._input_stream(lib, 0x1234):
        assert calls == [(0x1234, 1)]
    assert calls[-1] == (None, 0)
    calls.clear()
    try:
        with engine._input_stream(lib, 0x10):
            raise RuntimeError("inside")
    except RuntimeError:
        pass
    assert calls == [(0x10, 1), (None, 0)]
    # the real library accepts the setting on a host without a GPU
    from gcolor_amd import _native as nat
    real = nat.load()
    assert real.gc_set_input_stream(ctypes.c_void_p(0), 0) == 0
