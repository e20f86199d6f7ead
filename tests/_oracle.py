"""ctypes binding of oracle/liboracle.so (the CPU restatement checker)."""
import ctypes
import pathlib
import subprocess

import numpy as np

ROOT = pathlib.Path(__file__).resolve().parents[1]
LIB = ROOT / "oracle" / "liboracle.so"


class Info(ctypes.Structure):
    _fields_ = [("frame_bytes", ctypes.c_int), ("channels", ctypes.c_int), ("hz", ctypes.c_int),
                ("layer", ctypes.c_int), ("bitrate_kbps", ctypes.c_int)]


_lib = None


def lib():
    global _lib
    if _lib is None:
        if not LIB.exists():
            subprocess.check_call(["make", "-s", "-C", str(ROOT / "oracle")])
        L = ctypes.CDLL(str(LIB))
        L.orc_create.restype = ctypes.c_void_p
        L.orc_destroy.argtypes = [ctypes.c_void_p]
        L.orc_decode_frame.argtypes = [ctypes.c_void_p, ctypes.c_char_p, ctypes.c_int, ctypes.c_void_p,
                                       ctypes.POINTER(Info)]
        L.orc_get_taps.argtypes = [ctypes.c_void_p] + [ctypes.c_void_p] * 4
        L.orc_decode_stream.argtypes = [ctypes.c_char_p, ctypes.c_long, ctypes.c_void_p, ctypes.c_long,
                                        ctypes.POINTER(ctypes.c_int), ctypes.POINTER(ctypes.c_int)]
        L.orc_decode_stream.restype = ctypes.c_long
        L.orc_decode_stream_n.argtypes = [ctypes.c_char_p, ctypes.c_long, ctypes.c_void_p, ctypes.c_long,
                                          ctypes.POINTER(ctypes.c_int), ctypes.POINTER(ctypes.c_int),
                                          ctypes.POINTER(ctypes.c_long)]
        L.orc_decode_stream_n.restype = ctypes.c_long
        L.orc_decode_stream_opts.argtypes = L.orc_decode_stream_n.argtypes + [ctypes.c_int]
        L.orc_decode_stream_opts.restype = ctypes.c_long
        L.orc_set_options.argtypes = [ctypes.c_void_p, ctypes.c_int]
        L.orc_is_info_frame.argtypes = [ctypes.c_char_p, ctypes.c_long]
        L.orc_synth_only.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                     ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p]
        L.orc_skip_id3v2.argtypes = [ctypes.c_char_p, ctypes.c_long]
        L.orc_skip_id3v2.restype = ctypes.c_long
        L.orc_parse_info_tag.argtypes = [ctypes.c_char_p, ctypes.c_long, ctypes.c_void_p]
        _lib = L
    return _lib


def info_tag(data: bytes):
    """(found, dict) of the stream's leading Xing/Info + LAME tag (gapless)."""
    out = np.zeros(6, np.int32)
    found = lib().orc_parse_info_tag(data, len(data), out.ctypes.data)
    keys = ("has_lame", "enc_delay", "enc_padding", "total_frames", "skip_samples")
    d = dict(zip(keys, (int(x) for x in out)))
    spf = int(out[5])  # samples per frame: 1152, or 576 for MPEG-2/2.5
    d["end_sample"] = d["total_frames"] * spf + 529 - d["enc_padding"] if d["has_lame"] and d["total_frames"] > 0 else -1
    return bool(found), d


OPT_CRC_CHECK = 1  # ORC_OPT_CRC_CHECK: drop frames whose CRC-16 mismatches


def decode_stream(data: bytes, max_frames=100000, opts=0):
    """Planar float32 [nch, samples] (ID3v2 and Xing/Info frame skipped;
    1152 samples per MPEG-1 frame, 576 per MPEG-2/2.5 frame)."""
    L = lib()
    out = np.zeros((2, max_frames * 1152), np.float32)
    nch, hz, ns = ctypes.c_int(), ctypes.c_int(), ctypes.c_long()
    L.orc_decode_stream_opts(data, len(data), out.ctypes.data, max_frames, ctypes.byref(nch), ctypes.byref(hz),
                             ctypes.byref(ns), int(opts))
    return out[: nch.value, : ns.value], hz.value


class Decoder:
    """Per-frame oracle decoder with parity taps."""

    def __init__(self, opts=0):
        self.L = lib()
        self.d = self.L.orc_create()
        self.L.orc_set_options(self.d, int(opts))

    def __del__(self):
        try:
            self.L.orc_destroy(self.d)
        except Exception:
            pass

    def decode_frame(self, frame: bytes):
        pcm = np.zeros((2, 1152), np.float32)
        info = Info()
        r = self.L.orc_decode_frame(self.d, frame, len(frame), pcm.ctypes.data, ctypes.byref(info))
        return r, pcm[: info.channels], info

    def taps(self):
        is_ = np.zeros((2, 2, 576), np.int16)
        sf = np.zeros((2, 2, 40), np.uint8)
        xr = np.zeros((2, 2, 576), np.float32)
        side = np.zeros((2, 2, 20), np.int32)
        self.L.orc_get_taps(self.d, is_.ctypes.data, sf.ctypes.data, xr.ctypes.data, side.ctypes.data)
        return is_, sf, xr, side
