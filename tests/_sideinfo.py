"""Independent pure-Python walk of MPEG-1 Layer III frames and side info (test
helper; ISO/IEC 11172-3 2.4.1.3 header, 2.4.1.7 side info).

It shares no code or tables with the product (mp3d_tables.h) or the oracle:
the long-band edges below are SURVEY.md Appendix A.3's ISO values.  Used to
state what the FFmpeg-pinned fixtures cover (tests/test_golden_coverage.py).
"""

BITRATE = [0, 32, 40, 48, 56, 64, 80, 96, 112, 128, 160, 192, 224, 256, 320]
HZ = [44100, 48000, 32000]
SFB_LONG = {
    44100: [0, 4, 8, 12, 16, 20, 24, 30, 36, 44, 52, 62, 74, 90, 110, 134, 162, 196, 238, 288, 342, 418, 576],
    48000: [0, 4, 8, 12, 16, 20, 24, 30, 36, 42, 50, 60, 72, 88, 106, 128, 156, 190, 230, 276, 330, 384, 576],
    32000: [0, 4, 8, 12, 16, 20, 24, 30, 36, 44, 54, 66, 82, 102, 126, 156, 194, 240, 296, 364, 448, 550, 576],
}


class _Bits:
    def __init__(self, b):
        self.b, self.p = b, 0

    def get(self, n):
        v = 0
        for _ in range(n):
            v = (v << 1) | ((self.b[self.p >> 3] >> (7 - (self.p & 7))) & 1)
            self.p += 1
        return v


def frames(data: bytes):
    """Yield (offset, header dict) of each MPEG-1 Layer III frame of a
    generator stream (frames back to back from offset 0, no tags)."""
    pos = 0
    while pos + 4 <= len(data):
        b1, b2, b3 = data[pos + 1], data[pos + 2], data[pos + 3]
        assert data[pos] == 0xFF and (b1 & 0xE0) == 0xE0, pos
        if (b1 >> 3) & 3 != 3:  # not MPEG-1: outside this helper's scope
            return
        br, sr, pad = b2 >> 4, (b2 >> 2) & 3, (b2 >> 1) & 1
        hz = HZ[sr]
        n = 144000 * BITRATE[br] // hz + pad
        yield pos, dict(kbps=BITRATE[br], hz=hz, crc=not (b1 & 1), mode=b3 >> 6, mode_ext=(b3 >> 4) & 3,
                        frame_bytes=n)
        pos += n


def side_info(data: bytes, off: int, h: dict):
    """MPEG-1 side info of the frame at `off`: dict with main_data_begin,
    scfsi and units[gr][ch] (ISO 2.4.1.7 field names)."""
    nch = 1 if h["mode"] == 3 else 2
    bits = _Bits(data[off + 4 + (2 if h["crc"] else 0):])
    s = dict(main_data_begin=bits.get(9))
    bits.get(5 if nch == 1 else 3)
    s["scfsi"] = [bits.get(4) for _ in range(nch)]
    units = []
    for gr in range(2):
        row = []
        for ch in range(nch):
            u = dict(part2_3_length=bits.get(12), big_values=bits.get(9), global_gain=bits.get(8),
                     scalefac_compress=bits.get(4), window_switching=bits.get(1))
            if u["window_switching"]:
                u.update(block_type=bits.get(2), mixed=bits.get(1), table_select=[bits.get(5), bits.get(5), 0],
                         subblock_gain=[bits.get(3) for _ in range(3)])
            else:
                u.update(block_type=0, mixed=0, table_select=[bits.get(5) for _ in range(3)],
                         subblock_gain=[0, 0, 0], region0_count=bits.get(4), region1_count=bits.get(3))
            u.update(preflag=bits.get(1), scalefac_scale=bits.get(1), count1table_select=bits.get(1))
            row.append(u)
        units.append(row)
    s["units"] = units
    return s


def used_tables(u: dict, hz: int):
    """Huffman tables of the unit's non-empty big_values regions (ISO
    2.4.2.7: window switching -> region0 = 36 lines, region1 = the rest, no
    region2; else region edges at the long bands region0_count + 1 and
    region0_count + region1_count + 2), each clamped to 2 * big_values."""
    end = 2 * u["big_values"]
    if u["window_switching"]:
        r1, r2 = 36, 576
    else:
        sfb = SFB_LONG[hz]
        r1 = sfb[min(u["region0_count"] + 1, 22)]
        r2 = sfb[min(u["region0_count"] + u["region1_count"] + 2, 22)]
    r1, r2 = min(r1, end), min(r2, end)
    out = set()
    for lo, hi, t in ((0, r1, u["table_select"][0]), (r1, r2, u["table_select"][1]), (r2, end, u["table_select"][2])):
        if hi > lo:
            out.add(t)
    return out
