"""What the FFmpeg-pinned fixtures cover (VERDICT r02 "do this" 1).

Every MPEG-1 golden stream is walked by an independent Python side-info
parser (tests/_sideinfo.py: no code or table shared with the product or the
oracle) and the union of what it exercises is asserted: every Huffman table
ISO defines (incl. 10, 16-18, 20-23, which the real keypress file never
selects) in a non-empty big_values region, every block type and mixed
blocks, main_data_begin over 0..511, both count1 tables, every channel mode
and intensity / M/S combination, all three MPEG-1 rates, CRC-protected
frames, every bitrate index, and at BASELINE-config scale: the bench's own
C3 / C5 streams and >= 256 frames per C5 class."""
import collections

import _golden
import _sideinfo as si


def _walk():
    m = _golden.manifest()
    cov = collections.defaultdict(collections.Counter)
    frames_by_case = {}
    for name in sorted(m):
        if name.startswith(("lsf_", "edge_")):
            continue  # LSF (own walk) and edited streams
        data, _ = _golden.case(name)
        if name.startswith("keypress"):
            data = data[m[name]["tagless_offset"]:]
        n = 0
        for off, h in si.frames(data):
            n += 1
            s = si.side_info(data, off, h)
            mdb = s["main_data_begin"]
            cov["mdb"][mdb] += 1
            cov["mode"][(h["mode"], h["mode_ext"] if h["mode"] == 1 else 0)] += 1
            cov["hz"][h["hz"]] += 1
            cov["kbps"][h["kbps"]] += 1
            cov["crc"][h["crc"]] += 1
            cov["scfsi"][any(s["scfsi"])] += 1
            for row in s["units"]:
                for u in row:
                    for t in si.used_tables(u, h["hz"]):
                        cov["table"][t] += 1
                    cov["block"][(u["block_type"], u["mixed"])] += 1
                    cov["count1"][u["count1table_select"]] += 1
                    cov["sbg"][any(u["subblock_gain"])] += 1
                    cov["preflag"][u["preflag"]] += 1
                    cov["sfs"][u["scalefac_scale"]] += 1
        frames_by_case[name] = n
    return cov, frames_by_case


def test_ffmpeg_pinned_set_covers_the_bitstream_syntax():
    cov, _ = _walk()
    iso_tables = set(range(32)) - {4, 14}  # 4 and 14 are not defined by ISO
    assert set(cov["table"]) == iso_tables
    assert min(cov["table"][t] for t in iso_tables) >= 100  # each table in >= 100 units
    assert set(cov["block"]) == {(0, 0), (1, 0), (2, 0), (3, 0), (2, 1)}
    assert min(cov["mdb"]) == 0 and max(cov["mdb"]) == 511
    assert cov["mdb"][511] >= 100 and sum(c for v, c in cov["mdb"].items() if v >= 256) >= 1000
    assert set(cov["count1"]) == {0, 1}
    for k in ("sbg", "preflag", "sfs", "scfsi", "crc"):
        assert cov[k][True] >= 100 and cov[k][False] >= 100, k
    # mono, stereo, dual channel, joint stereo with every mode_extension
    assert set(cov["mode"]) == {(3, 0), (0, 0), (2, 0), (1, 0), (1, 1), (1, 2), (1, 3)}
    assert set(cov["hz"]) == {32000, 44100, 48000}
    assert set(cov["kbps"]) == set(si.BITRATE[1:])


def test_ffmpeg_pinned_set_at_baseline_scale():
    _, n = _walk()
    # the bench's own C3 streams (global ids 0..7) and C5 streams (0..3), 32 frames each
    assert all(n["bench_c3_g%d" % g] == 32 for g in range(8))
    assert all(n["bench_c5_g%d" % g] == 32 for g in range(4))
    classes = [k for k in n if k.startswith("scale_")]
    assert len(classes) >= 6 and all(n[k] >= 256 for k in classes)
    assert n["long_c3_512"] == 512
    assert sum(n.values()) >= 3000
