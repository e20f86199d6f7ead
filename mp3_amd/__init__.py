"""mp3_amd -- MI355X-native batched MPEG-1 Layer III decoder (Python host side).

Mirrors the C ABI of include/mp3d.h (the drop-in boundary for the reference
player's per-frame decode call):

  Decoder       per-frame decode (mp3d_decode_frame): bytes -> int16 PCM
  BatchDecoder  many concurrent streams on one GPU (mp3d_batch_*), inputs and
                outputs as numpy arrays (host) or torch tensors (device)

The compute path is the HIP library mp3_amd/libmp3d.so; there is no CPU
fallback.  Importing works without a GPU; creating a decoder does not.
"""
import ctypes
import os
import pathlib

import numpy as np

_HERE = pathlib.Path(__file__).resolve().parent
LIB_PATH = pathlib.Path(os.environ["MP3D_LIB"]) if os.environ.get("MP3D_LIB") else _HERE / "libmp3d.so"

MP3D_E = {0: "ok", -1: "bad argument", -2: "no usable HIP device", -3: "HIP runtime error", -4: "out of memory",
          -5: "batch exceeds handle capacity", -6: "no complete frame in buffer"}


class FrameInfo(ctypes.Structure):
    _fields_ = [("frame_bytes", ctypes.c_int), ("channels", ctypes.c_int), ("hz", ctypes.c_int),
                ("layer", ctypes.c_int), ("bitrate_kbps", ctypes.c_int), ("samples", ctypes.c_int)]


class StreamInfo(ctypes.Structure):
    """mp3d_stream_info: leading Xing/Info tag and FFmpeg-style gapless trim."""
    _fields_ = [("has_tag", ctypes.c_int), ("has_lame", ctypes.c_int), ("enc_delay", ctypes.c_int),
                ("enc_padding", ctypes.c_int), ("total_frames", ctypes.c_int), ("skip_samples", ctypes.c_int),
                ("end_sample", ctypes.c_longlong)]

    def as_dict(self):
        return {k: getattr(self, k) for k, _ in self._fields_}


FRAME_INFO_DT = np.dtype([("frame_bytes", np.int32), ("channels", np.int32), ("hz", np.int32),
                          ("layer", np.int32), ("bitrate_kbps", np.int32), ("samples", np.int32)])

EXPORTS = ["mp3d_dec_create", "mp3d_dec_create_on", "mp3d_dec_destroy", "mp3d_dec_reset", "mp3d_decode_frame",
           "mp3d_decode_frame_f32", "mp3d_batch_decode_f32",
           "mp3d_batch_create", "mp3d_batch_destroy", "mp3d_batch_reset", "mp3d_batch_decode", "mp3d_batch_sync",
           "mp3d_batch_huffman_only", "mp3d_batch_synth_only", "mp3d_strerror", "mp3d_last_hip_error",
           "mp3d_abi_version", "mp3d_batch_set_timing", "mp3d_batch_kernel_times", "mp3d_batch_stream_info",
           "mp3d_dec_stream_info", "mp3d_batch_decode_long",
           "mp3d_long_plan", "mp3d_batch_set_options", "mp3d_dec_set_options", "mp3d_decode_frame_ex",
           "mp3d_state_bytes", "mp3d_batch_get_state", "mp3d_batch_set_state", "mp3d_dec_get_state",
           "mp3d_dec_set_state"]

OPT_CRC_CHECK = 1  # MP3D_OPT_CRC_CHECK: drop frames whose CRC-16 mismatches
FRAME_F32, FRAME_LAST = 1, 2  # mp3d_decode_frame_ex flags

_lib = None


class MP3DError(RuntimeError):
    pass


def lib():
    """Load libmp3d.so (fails loudly if it was not built)."""
    global _lib
    if _lib is None:
        if not LIB_PATH.exists():
            raise ImportError("mp3_amd: %s missing -- run __graft_entry__.build() (no CPU fallback exists)" % LIB_PATH)
        L = ctypes.CDLL(str(LIB_PATH))
        vp, i, u64p, u32p = ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p
        L.mp3d_dec_create.argtypes = [ctypes.POINTER(vp)]
        L.mp3d_dec_create_on.argtypes = [i, ctypes.POINTER(vp)]
        L.mp3d_dec_destroy.argtypes = [vp]
        L.mp3d_dec_destroy.restype = None
        L.mp3d_dec_reset.argtypes = [vp]
        L.mp3d_dec_reset.restype = None
        L.mp3d_decode_frame.argtypes = [vp, ctypes.c_char_p, ctypes.c_size_t, vp, ctypes.POINTER(FrameInfo)]
        L.mp3d_batch_create.argtypes = [i, i, i, ctypes.POINTER(vp)]
        L.mp3d_batch_destroy.argtypes = [vp]
        L.mp3d_batch_destroy.restype = None
        L.mp3d_batch_reset.argtypes = [vp]
        L.mp3d_batch_decode.argtypes = [vp, vp, u64p, u32p, i, i, vp, vp, vp]
        L.mp3d_batch_decode_f32.argtypes = [vp, vp, u64p, u32p, i, i, vp, vp, vp]
        L.mp3d_decode_frame_f32.argtypes = [vp, ctypes.c_char_p, ctypes.c_size_t, vp, ctypes.POINTER(FrameInfo)]
        L.mp3d_batch_sync.argtypes = [vp]
        L.mp3d_batch_huffman_only.argtypes = [vp, vp, u64p, u32p, i, i, vp, vp, vp]
        L.mp3d_batch_synth_only.argtypes = [vp, vp, vp, vp, i, i, i, i, vp, vp]
        L.mp3d_strerror.argtypes = [i]
        L.mp3d_strerror.restype = ctypes.c_char_p
        L.mp3d_batch_set_timing.argtypes = [vp, i]
        L.mp3d_batch_kernel_times.argtypes = [vp, vp]
        L.mp3d_batch_stream_info.argtypes = [vp, i, vp]
        L.mp3d_dec_stream_info.argtypes = [vp, ctypes.POINTER(StreamInfo)]
        L.mp3d_batch_decode_long.argtypes = [vp, vp, ctypes.c_size_t, i, vp, i, ctypes.c_longlong, vp,
                                             ctypes.POINTER(ctypes.c_longlong), ctypes.POINTER(StreamInfo)]
        L.mp3d_long_plan.argtypes = [ctypes.c_char_p, ctypes.c_size_t, i, ctypes.c_longlong, vp, vp,
                                     ctypes.POINTER(ctypes.c_longlong), ctypes.POINTER(ctypes.c_int)]
        L.mp3d_batch_set_options.argtypes = [vp, i]
        L.mp3d_dec_set_options.argtypes = [vp, i]
        L.mp3d_decode_frame_ex.argtypes = [vp, ctypes.c_char_p, ctypes.c_size_t, vp, i, ctypes.POINTER(FrameInfo)]
        L.mp3d_state_bytes.restype = ctypes.c_size_t
        L.mp3d_batch_get_state.argtypes = [vp, i, i, vp]
        L.mp3d_batch_set_state.argtypes = [vp, i, i, vp]
        L.mp3d_dec_get_state.argtypes = [vp, vp]
        L.mp3d_dec_set_state.argtypes = [vp, vp]
        _lib = L
    return _lib


def _check(rc):
    if rc < 0:
        L = lib()
        raise MP3DError("mp3d error %d (%s), hip error %d" % (rc, L.mp3d_strerror(rc).decode(), L.mp3d_last_hip_error()))
    return rc


def _ptr(x):
    """(pointer, keepalive) for a numpy array, torch tensor, bytes or None."""
    if x is None:
        return None, None
    if isinstance(x, (bytes, bytearray)):
        a = np.frombuffer(bytes(x), np.uint8)
        return a.ctypes.data, a
    if isinstance(x, np.ndarray):
        if not x.flags.c_contiguous:
            raise ValueError("array must be C-contiguous")
        return x.ctypes.data, x
    if hasattr(x, "data_ptr"):
        if not x.is_contiguous():
            raise ValueError("tensor must be contiguous")
        return x.data_ptr(), x
    raise TypeError("unsupported buffer type %r" % type(x))


class Decoder:
    """Per-frame decoder (mp3d_decode_frame), one per stream."""

    def __init__(self, device=None):
        L = lib()
        h = ctypes.c_void_p()
        if device is None:
            _check(L.mp3d_dec_create(ctypes.byref(h)))
        else:
            _check(L.mp3d_dec_create_on(int(device), ctypes.byref(h)))
        self._h = h

    def close(self):
        if getattr(self, "_h", None):
            lib().mp3d_dec_destroy(self._h)
            self._h = None

    __del__ = close

    def reset(self):
        lib().mp3d_dec_reset(self._h)

    def set_options(self, flags):
        """MP3D_OPT_* flags (OPT_CRC_CHECK) for later decode calls."""
        _check(lib().mp3d_dec_set_options(self._h, int(flags)))

    def decode_frame(self, buf, f32=False, last=False):
        """Returns (samples_per_channel, pcm [samples*channels], FrameInfo);
        pcm is int16, or float32 (full scale 1.0, unclipped) with f32=True.
        last=True: buf holds the rest of the stream, so a final frame cut
        short decodes with its missing bytes as zeros (MP3D_FRAME_LAST)."""
        pcm = np.zeros(2304, np.float32 if f32 else np.int16)
        info = FrameInfo()
        buf = bytes(buf)
        flags = (FRAME_F32 if f32 else 0) | (FRAME_LAST if last else 0)
        n = _check(lib().mp3d_decode_frame_ex(self._h, buf, len(buf), pcm.ctypes.data, flags, ctypes.byref(info)))
        return n, pcm[: n * max(info.channels, 1)], info

    def get_state(self):
        """Opaque decoder state (np.uint8 [state_bytes()]) for set_state."""
        buf = np.zeros(state_bytes(), np.uint8)
        _check(lib().mp3d_dec_get_state(self._h, buf.ctypes.data))
        return buf

    def set_state(self, buf):
        buf = np.ascontiguousarray(buf, np.uint8)
        if buf.size != state_bytes():
            raise ValueError("state blob of %d bytes, expected %d" % (buf.size, state_bytes()))
        _check(lib().mp3d_dec_set_state(self._h, buf.ctypes.data))

    def stream_info(self):
        """StreamInfo of the stream decoded so far (Xing/Info tag, gapless)."""
        info = StreamInfo()
        _check(lib().mp3d_dec_stream_info(self._h, ctypes.byref(info)))
        return info

    def decode_stream(self, data, gapless=False, f32=False):
        """Decode a whole byte stream; returns int16 (float32 with f32=True)
        [channels, samples].  gapless=True drops encoder delay / padding as
        the stream's LAME tag says (gapless_trim)."""
        if gapless:
            return gapless_trim(self.decode_stream(data, f32=f32), self.stream_info())
        data = bytes(data)
        pos, out, nch = 0, [], 0
        while pos < len(data):
            try:
                n, pcm, info = self.decode_frame(data[pos:], f32=f32, last=True)
            except MP3DError:
                break
            if info.frame_bytes <= 0:
                break
            pos += info.frame_bytes
            if n:
                nch = info.channels
                out.append(pcm.reshape(n, nch))
        if not out:
            return np.zeros((0, 0), np.float32 if f32 else np.int16)
        return np.concatenate(out).T.copy()


class BatchDecoder:
    """Batched decoder: per-stream state stays in HBM across calls."""

    def __init__(self, max_streams, max_frames, device=0):
        L = lib()
        h = ctypes.c_void_p()
        _check(L.mp3d_batch_create(int(device), int(max_streams), int(max_frames), ctypes.byref(h)))
        self._h = h
        self.device = device
        self.max_streams, self.max_frames = max_streams, max_frames

    def close(self):
        if getattr(self, "_h", None):
            lib().mp3d_batch_destroy(self._h)
            self._h = None

    __del__ = close

    def reset(self):
        _check(lib().mp3d_batch_reset(self._h))

    def set_options(self, flags):
        """MP3D_OPT_* flags (OPT_CRC_CHECK) for later decode calls."""
        _check(lib().mp3d_batch_set_options(self._h, int(flags)))

    def sync(self):
        _check(lib().mp3d_batch_sync(self._h))

    def set_timing(self, on=True):
        _check(lib().mp3d_batch_set_timing(self._h, int(on)))

    def kernel_times_us(self):
        t = np.zeros(3, np.float32)
        _check(lib().mp3d_batch_kernel_times(self._h, t.ctypes.data))
        return dict(zip(("demux", "huffman", "synth"), t.tolist()))

    @staticmethod
    def _geom(offsets, sizes):
        off = np.ascontiguousarray(offsets, dtype=np.uint64)
        sz = np.ascontiguousarray(sizes, dtype=np.uint32)
        if off.shape != sz.shape:
            raise ValueError("offsets/sizes shape mismatch")
        return off, sz

    def decode(self, frames, offsets, sizes, frames_per_stream, pcm=None, infos=None, stream=None, f32=False):
        """frames: bytes/np.uint8/torch.uint8; pcm: None (allocate host) or
        int16 (float32 with f32=True) array/tensor [n, F, 2304]; infos: None
        or FRAME_INFO_DT array / int32 tensor [n, F, 6].  Returns (pcm, infos)."""
        off, sz = self._geom(offsets, sizes)
        n, F = off.size, int(frames_per_stream)
        if pcm is None:
            pcm = np.zeros((n, F, 2304), np.float32 if f32 else np.int16)
        if infos is None:
            infos = np.zeros((n, F), FRAME_INFO_DT)
        fp, k1 = _ptr(frames)
        pp, k2 = _ptr(pcm)
        ip, k3 = _ptr(infos)
        fn = lib().mp3d_batch_decode_f32 if f32 else lib().mp3d_batch_decode
        _check(fn(self._h, fp, off.ctypes.data, sz.ctypes.data, n, F, pp, ip, ctypes.c_void_p(stream) if stream else None))
        return pcm, infos

    @staticmethod
    def _nbytes(x):
        """Byte size of a contiguous host array / device tensor (its element
        count times element size, whatever the dtype)."""
        if hasattr(x, "numel"):
            if not x.is_contiguous():
                raise ValueError("state tensor must be contiguous")
            return x.numel() * x.element_size()
        if not isinstance(x, np.ndarray) or not x.flags.c_contiguous:
            raise ValueError("state buffer must be a C-contiguous numpy array or tensor")
        return x.nbytes

    def _state_range(self, first, n):
        first, n = int(first), int(n)
        if first < 0 or n <= 0 or first + n > self.max_streams:
            raise ValueError("streams [%d, %d) outside the handle's %d" % (first, first + n, self.max_streams))
        return first, n

    def get_state(self, first=0, n=None, out=None):
        """State blobs of streams [first, first + n): np.uint8 [n, state_bytes()]
        (or into `out`, a host array or device tensor of exactly that many
        bytes)."""
        first, n = self._state_range(first, self.max_streams - int(first) if n is None else n)
        if out is None:
            out = np.zeros((n, state_bytes()), np.uint8)
        if self._nbytes(out) != n * state_bytes():
            raise ValueError("out holds %d bytes, %d streams need %d" % (self._nbytes(out), n, n * state_bytes()))
        op, k = _ptr(out)
        _check(lib().mp3d_batch_get_state(self._h, first, n, op))
        return out

    def set_state(self, buf, first=0):
        """Restore state blobs [n, state_bytes()] into streams [first, first + n);
        buf is a contiguous host array or device tensor of n * state_bytes()
        bytes (any dtype: the byte count decides n)."""
        if not hasattr(buf, "numel"):
            buf = np.asarray(buf)
            if not buf.flags.c_contiguous:
                raise ValueError("state buffer must be C-contiguous")
        nb = self._nbytes(buf)
        if nb == 0 or nb % state_bytes():
            raise ValueError("state buffer of %d bytes is not a whole number of %d-byte blobs" % (nb, state_bytes()))
        first, n = self._state_range(first, nb // state_bytes())
        bp, k = _ptr(buf)
        _check(lib().mp3d_batch_set_state(self._h, first, n, bp))

    def stream_info(self, n_streams):
        """[StreamInfo] of the first n_streams streams (after a decode call)."""
        arr = (StreamInfo * int(n_streams))()
        _check(lib().mp3d_batch_stream_info(self._h, int(n_streams), ctypes.cast(arr, ctypes.c_void_p)))
        return list(arr)

    def decode_long(self, data, segment_frames=32, max_frames=None, pcm=None, infos=None, f32=False):
        """Frame-parallel decode of ONE long stream (mp3d_batch_decode_long):
        segments of segment_frames output frames run as concurrent virtual
        streams, bit-identical to a sequential decode.  data: bytes /
        np.uint8 / torch.uint8 (host or device).  pcm: None (allocate host)
        or [max_frames, 2304] int16 (float32 with f32=True) array/tensor.
        Returns (pcm[:n], infos[:n], StreamInfo)."""
        nbytes = data.numel() if hasattr(data, "numel") else len(data)
        if max_frames is None:
            if pcm is not None or infos is not None:
                max_frames = min(len(x) for x in (pcm, infos) if x is not None)
            else:  # exact: the host frame walk of the plan
                host = data.cpu().numpy().tobytes() if hasattr(data, "cpu") else bytes(data)
                max_frames = len(long_plan(host, segment_frames, max_frame_slots(nbytes))[0])
        for x in (pcm, infos):
            if x is not None and len(x) < max_frames:
                raise ValueError("pcm / infos hold %d rows < max_frames %d" % (len(x), max_frames))
        max_frames = max(1, int(max_frames))
        if pcm is None:
            pcm = np.zeros((max_frames, 2304), np.float32 if f32 else np.int16)
        if infos is None:
            infos = np.zeros(max_frames, FRAME_INFO_DT)
        dp, k1 = _ptr(data)
        pp, k2 = _ptr(pcm)
        ip, k3 = _ptr(infos)
        n = ctypes.c_longlong()
        si = StreamInfo()
        _check(lib().mp3d_batch_decode_long(self._h, dp, nbytes, int(segment_frames), pp, int(f32), int(max_frames),
                                            ip, ctypes.byref(n), ctypes.byref(si)))
        return pcm[: n.value], infos[: n.value], si

    def huffman_only(self, frames, offsets, sizes, frames_per_stream):
        off, sz = self._geom(offsets, sizes)
        n, F = off.size, int(frames_per_stream)
        is_out = np.zeros((n, F, 2, 2, 576), np.int16)
        sf_out = np.zeros((n, F, 2, 2, 40), np.uint8)
        fp, k1 = _ptr(frames)
        _check(lib().mp3d_batch_huffman_only(self._h, fp, off.ctypes.data, sz.ctypes.data, n, F,
                                             is_out.ctypes.data, sf_out.ctypes.data, None))
        return is_out, sf_out

    def synth_only(self, xr, block_type, mixed, nch, hz, pcm=None, stream=None):
        """xr f32 [n, F, 2, nch, 576]; block_type/mixed uint8 [n, F, 2, nch]."""
        n, F = int(xr.shape[0]), int(xr.shape[1])
        if pcm is None:
            pcm = np.zeros((n, F, 2304), np.int16)
        xp, k1 = _ptr(xr)
        bp, k2 = _ptr(block_type)
        mp, k3 = _ptr(mixed)
        pp, k4 = _ptr(pcm)
        _check(lib().mp3d_batch_synth_only(self._h, xp, bp, mp, n, F, int(nch), int(hz), pp,
                                           ctypes.c_void_p(stream) if stream else None))
        return pcm


def state_bytes():
    """Bytes of one stream's opaque decoder state (mp3d_state_bytes)."""
    return int(lib().mp3d_state_bytes())


def max_frame_slots(nbytes):
    """Upper bound on the frame slots in nbytes of stream: the smallest
    Layer III frame is 24 B (MPEG-2 LSF, 8 kbps at 24 kHz; MPEG-1: 96 B)."""
    return int(nbytes) // 24 + 2


def long_plan(data, segment_frames=32, max_frames=None):
    """Host-side segment plan of BatchDecoder.decode_long (mp3d_long_plan;
    no GPU needed).  Returns (frame_off [n] uint64, seg_start [K] int64,
    max_warmup)."""
    data = bytes(data)
    if max_frames is None:
        max_frames = max_frame_slots(len(data))
    L = int(segment_frames)
    off = np.zeros(max_frames, np.uint64)
    seg = np.zeros(max_frames // max(L, 1) + 2, np.int64)
    n, w = ctypes.c_longlong(), ctypes.c_int()
    _check(lib().mp3d_long_plan(data, len(data), L, int(max_frames), off.ctypes.data, seg.ctypes.data,
                                ctypes.byref(n), ctypes.byref(w)))
    k = (n.value + L - 1) // L
    return off[: n.value], seg[:k], w.value


def pcm_to_planar(pcm_frames, infos):
    """[F, 2304] int16/float32 + infos [F] -> [channels, samples] for frames
    with audio (1152 samples per channel, 576 for an MPEG-2 / 2.5 LSF frame,
    interleaved at the start of the frame's row)."""
    rows = []
    nch = 0
    for f in range(pcm_frames.shape[0]):
        n = int(infos[f]["samples"])
        if n:
            nch = int(infos[f]["channels"])
            rows.append(pcm_frames[f, : n * nch].reshape(n, nch))
    if not rows:
        return np.zeros((0, 0), pcm_frames.dtype)
    return np.concatenate(rows).T.copy()


def gapless_trim(planar, info):
    """Apply a stream's gapless trim (StreamInfo or its dict) to planar PCM
    [channels, samples] holding every decoded sample from the stream start:
    FFmpeg semantics (libavformat/mp3dec.c) -- drop the first skip_samples,
    and everything from end_sample on when the tag gives a frame count."""
    get = info.get if isinstance(info, dict) else (lambda k: getattr(info, k))
    if not get("has_lame"):
        return planar
    end = get("end_sample")
    stop = planar.shape[1] if end is None or end < 0 else min(int(end), planar.shape[1])
    return planar[:, int(get("skip_samples")):stop]
