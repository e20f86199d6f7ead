"""The C-ABI library loads and exports every symbol include/mp3d.h declares
(no compute calls: this runs on CPU-only machines too)."""
import ctypes
import re

import mp3_amd
from mp3_amd import _build

HDR = _build.ROOT / "include" / "mp3d.h"


def declared():
    src = HDR.read_text()
    return sorted(set(re.findall(r"MP3D_API\s+[\w\s\*]*?\b(mp3d_\w+)\s*\(", src)))


def test_header_declares_api():
    names = declared()
    assert "mp3d_decode_frame" in names and "mp3d_batch_decode" in names
    assert len(names) == len(mp3_amd.EXPORTS)
    assert sorted(mp3_amd.EXPORTS) == names


def test_library_exports_all_declared_symbols():
    _build.build_hip()
    L = ctypes.CDLL(str(mp3_amd.LIB_PATH))
    for n in declared():
        assert hasattr(L, n), n
    assert L.mp3d_abi_version() == 5
    assert mp3_amd.state_bytes() > 8000  # the opaque per-stream state blob


def test_no_device_fails_loudly_or_creates():
    """Without a GPU, creation must fail with MP3D_E_NO_DEVICE (no CPU fallback)."""
    import torch
    L = mp3_amd.lib()
    h = ctypes.c_void_p()
    rc = L.mp3d_batch_create(0, 1, 1, ctypes.byref(h))
    if torch.cuda.device_count() == 0:
        assert rc == -2
    else:
        assert rc == 0
        L.mp3d_batch_destroy(h)
