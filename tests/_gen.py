"""ctypes binding of the synthetic stream generator (mp3_amd/libmp3gen.so)."""
import ctypes
import pathlib

import numpy as np

ROOT = pathlib.Path(__file__).resolve().parents[1]


class GenCfg(ctypes.Structure):
    _fields_ = [(n, ctypes.c_int) for n in ("sr_idx", "bitrate_idx", "mode", "mode_ext", "short_pct",
                                              "mixed_pct", "crc_pct", "fill_pct", "max_reservoir")]


TRUTH_DT = np.dtype([("is", np.int16, 576), ("sf", np.uint8, 40), ("part2_3_length", np.int32),
                     ("big_values", np.int32), ("global_gain", np.int32), ("block_type", np.int32),
                     ("mixed", np.int32), ("count1", np.int32)])

# BASELINE.json configs -> generator settings
C3 = dict(sr_idx=0, bitrate_idx=9, mode=1, mode_ext=2, short_pct=5, mixed_pct=5, crc_pct=0, fill_pct=100,
          max_reservoir=511)
C5 = dict(sr_idx=-1, bitrate_idx=0, mode=-1, mode_ext=-1, short_pct=15, mixed_pct=25, crc_pct=30,
          fill_pct=100, max_reservoir=511)

_lib = None


def lib():
    global _lib
    if _lib is None:
        L = ctypes.CDLL(str(ROOT / "mp3_amd" / "libmp3gen.so"))
        L.mp3gen_stream.restype = ctypes.c_long
        L.mp3gen_stream.argtypes = [ctypes.POINTER(GenCfg), ctypes.c_uint64, ctypes.c_int, ctypes.c_void_p,
                                    ctypes.c_long, ctypes.c_void_p, ctypes.c_void_p]
        L.mp3gen_batch.restype = ctypes.c_long
        L.mp3gen_batch.argtypes = [ctypes.POINTER(GenCfg), ctypes.c_uint64, ctypes.c_int, ctypes.c_int,
                                   ctypes.c_void_p, ctypes.c_long, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int]
        L.mp3gen_max_bytes.restype = ctypes.c_long
        L.mp3gen_max_bytes.argtypes = [ctypes.POINTER(GenCfg), ctypes.c_int]
        assert L.mp3gen_truth_size() == TRUTH_DT.itemsize, (L.mp3gen_truth_size(), TRUTH_DT.itemsize)
        _lib = L
    return _lib


def stream(cfg: dict, seed: int, n_frames: int, truth=False):
    L = lib()
    c = GenCfg(**cfg)
    cap = L.mp3gen_max_bytes(ctypes.byref(c), n_frames)
    buf = np.zeros(cap, np.uint8)
    offs = np.zeros(n_frames, np.uint32)
    tr = np.zeros(n_frames * 4, TRUTH_DT) if truth else None
    n = L.mp3gen_stream(ctypes.byref(c), seed, n_frames, buf.ctypes.data, cap, offs.ctypes.data,
                        tr.ctypes.data if truth else None)
    assert n > 0
    out = bytes(buf[:n])
    return (out, offs, tr.reshape(n_frames, 2, 2)) if truth else (out, offs)


def batch(cfg: dict, seed_base: int, n_streams: int, n_frames: int, threads=8):
    L = lib()
    c = GenCfg(**cfg)
    cap = L.mp3gen_max_bytes(ctypes.byref(c), n_frames) * n_streams
    buf = np.empty(cap, np.uint8)
    offs = np.zeros(n_streams, np.uint64)
    sizes = np.zeros(n_streams, np.uint32)
    n = L.mp3gen_batch(ctypes.byref(c), seed_base, n_streams, n_frames, buf.ctypes.data, cap,
                       offs.ctypes.data, sizes.ctypes.data, threads)
    assert n > 0
    return buf[:n], offs, sizes
