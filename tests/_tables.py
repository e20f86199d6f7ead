"""Parse mp3_amd/csrc/mp3d_tables.h into numpy arrays (test helper).

The header is the single source of the ISO 11172-3 constants; tests read it
textually so that the CPU suite does not need a compiler for table checks.
"""
import pathlib
import re

import numpy as np

HDR = pathlib.Path(__file__).resolve().parents[1] / "mp3_amd" / "csrc" / "mp3d_tables.h"


def _strip_comments(s):
    s = re.sub(r"/\*.*?\*/", "", s, flags=re.S)
    return re.sub(r"//[^\n]*", "", s)


def load():
    src = _strip_comments(HDR.read_text())
    out = {}
    pat = re.compile(r"static const (\w+)\s+(?:\*const\s+)?(\w+)((?:\[[^\]]*\])+)\s*=\s*\{(.*?)\};", re.S)
    for m in pat.finditer(src):
        ctype, name, dims, body = m.groups()
        if ctype not in ("uint8_t", "int8_t", "uint16_t", "int32_t", "uint32_t", "double"):
            continue
        nums = re.findall(r"-?0x[0-9a-fA-F]+|-?\d+\.\d*|-?\d+", body)
        dt = {"uint8_t": np.uint8, "int8_t": np.int8, "uint16_t": np.uint16, "int32_t": np.int32,
              "uint32_t": np.uint32, "double": np.float64}[ctype]
        vals = [float(x) if dt is np.float64 else int(x, 0) for x in nums]
        shape = [int(d) for d in re.findall(r"\[(\d+)\]", dims)]
        arr = np.array(vals, dtype=dt)
        if shape and int(np.prod(shape)) == arr.size:
            arr = arr.reshape(shape)
        out[name] = arr
    return out


HTAB_ISO = [1, 2, 3, 5, 6, 7, 8, 9, 10, 11, 12, 13, 15, 16, 24]


def htab(t, iso_num):
    return t["MP3D_HCODE_%d" % iso_num], t["MP3D_HLEN_%d" % iso_num]
