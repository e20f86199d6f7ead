"""What the generator truth behind test_gpu_parity.test_huffman_bitexact_vs_truth
covers at the count1 edges (CPU; the GPU test then compares every unit).

k_huffman decodes count1 quadruples two per iteration from one window read
and stores each pair with one 16-B store; an unpaired last quadruple takes
an 8-B store, and a quadruple at line 572 is always unpaired (lines end at
576).  The parity batches must hold units with an odd and an even number of
quadruples, none, and count1 regions that run to the last line they can
reach: 576 after big_values regions of 2 big_values = 0 mod 4, 574 after
those of 2 mod 4 (a quadruple at 574 would pass line 576, so the loop stops
at k > 572)."""
import numpy as np
import pytest

import _gen

# the (cfg, seed) cases of test_gpu_parity.test_huffman_bitexact_vs_truth, n = 48 streams x F = 6 frames
CASES = [(_gen.C3, 101), (_gen.C5, 102), (_gen.C5, 103)]


def _units(cfg, seed, n=48, F=6):
    c1, bv2 = [], []
    for s in range(n):
        _, _, t = _gen.stream(cfg, seed + s, F, truth=True)
        c1.append(t["count1"].ravel())
        bv2.append(2 * t["big_values"].ravel())
    return np.concatenate(c1), np.concatenate(bv2)


@pytest.fixture(scope="module")
def units():
    c1, bv2 = zip(*(_units(cfg, seed) for cfg, seed in CASES))
    return np.concatenate(c1), np.concatenate(bv2)


def test_count1_pairing_edges_covered(units):
    c1, bv2 = units
    end = bv2 + 4 * c1
    assert ((c1 % 2) == 1).sum() >= 100, "odd quadruple counts (an unpaired last quadruple)"
    assert ((c1 % 2) == 0).sum() - (c1 == 0).sum() >= 100, "even quadruple counts (all paired)"
    assert (c1 == 0).sum() >= 10, "units without count1"
    assert (end <= 576).all()
    assert ((end == 576) & (bv2 % 4 == 0)).sum() >= 5, "count1 up to line 576"
    assert ((end == 574) & (bv2 % 4 == 2)).sum() >= 5, "count1 up to line 574 (the next quadruple would pass 576)"
