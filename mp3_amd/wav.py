"""WAV sink for decoded PCM (the player's output side).

write(path_or_file, planar, hz): planar [channels, samples] int16 ->
WAVE_FORMAT_PCM 16-bit, float32 -> WAVE_FORMAT_IEEE_FLOAT 32-bit (with the
'fact' chunk the format requires).  Host-side byte packing only; the samples
come from the GPU decoder (Decoder / BatchDecoder, int16 or f32 sinks)."""
import struct

import numpy as np


def wav_bytes(planar, hz):
    planar = np.asarray(planar)
    if planar.ndim != 2 or planar.shape[0] not in (1, 2):
        raise ValueError("planar PCM must be [channels (1 or 2), samples]")
    nch, n = planar.shape
    if planar.dtype == np.int16:
        fmt_tag, width = 1, 2
    elif planar.dtype == np.float32:
        fmt_tag, width = 3, 4
    else:
        raise TypeError("int16 or float32 PCM expected, got %s" % planar.dtype)
    data = np.ascontiguousarray(planar.T).astype(planar.dtype.newbyteorder("<")).tobytes()
    fmt = struct.pack("<HHIIHH", fmt_tag, nch, int(hz), int(hz) * nch * width, nch * width, 8 * width)
    chunks = [b"fmt " + struct.pack("<I", len(fmt)) + fmt]
    if fmt_tag == 3:
        chunks.append(b"fact" + struct.pack("<II", 4, n))
    chunks.append(b"data" + struct.pack("<I", len(data)) + data)
    body = b"WAVE" + b"".join(chunks)
    return b"RIFF" + struct.pack("<I", len(body)) + body


def write(path_or_file, planar, hz):
    blob = wav_bytes(planar, hz)
    if hasattr(path_or_file, "write"):
        path_or_file.write(blob)
    else:
        with open(path_or_file, "wb") as f:
            f.write(blob)
    return len(blob)


def read(path):
    """Minimal reader for files written by write(): (planar, hz)."""
    blob = open(path, "rb").read()
    assert blob[:4] == b"RIFF" and blob[8:12] == b"WAVE"
    pos, fmt, data = 12, None, None
    while pos + 8 <= len(blob):
        cid, size = blob[pos:pos + 4], struct.unpack("<I", blob[pos + 4:pos + 8])[0]
        body = blob[pos + 8:pos + 8 + size]
        if cid == b"fmt ":
            fmt = struct.unpack("<HHIIHH", body[:16])
        elif cid == b"data":
            data = body
        pos += 8 + size + (size & 1)
    tag, nch, hz = fmt[0], fmt[1], fmt[2]
    dt = np.dtype("<i2") if tag == 1 else np.dtype("<f4")
    return np.frombuffer(data, dt).reshape(-1, nch).T.astype(dt.newbyteorder("=")), hz
