"""Config 4's gather on the GPU: jpge_concat_segments (concat.hip), the pack of a
rank's .jpg bytes before its one transfer to rank 0 (jpgenc_amd/gather.py), against
numpy's concatenation of the same bytes."""
import numpy as np
import pytest

torch = pytest.importorskip("torch")
import jpgenc_amd as J  # noqa: E402

pytestmark = pytest.mark.gpu


def _check(lens, src_mis, dst_mis, seed=0):
    rng = np.random.default_rng(seed)
    dev = torch.device("cuda:0")
    pool = torch.from_numpy(rng.integers(0, 256, sum(lens) + 64 * len(lens) + 64, dtype=np.uint8)).to(dev)
    ptrs, want, pos = [], [], 0
    for k, n in enumerate(lens):
        pos += int(src_mis[k % len(src_mis)])
        ptrs.append(pool.data_ptr() + pos)
        want.append(pool[pos:pos + n].cpu().numpy())
        pos += n + 7
    tot = sum(lens)
    out = torch.full((tot + 64,), 0xA5, dtype=torch.uint8, device=dev)
    got_tot = J.concat_segments(0, 0, ptrs, lens, out.data_ptr() + dst_mis)
    torch.cuda.synchronize()
    assert got_tot == tot
    o = out.cpu().numpy()
    assert np.array_equal(o[dst_mis:dst_mis + tot], np.concatenate(want) if want else np.zeros(0, np.uint8))
    assert (o[:dst_mis] == 0xA5).all() and (o[dst_mis + tot:] == 0xA5).all()  # nothing outside the run


@pytest.mark.parametrize("dst_mis", [0, 1, 5, 15])
@pytest.mark.parametrize("src_mis", [(0,), (3,), (1, 14, 0, 7, 9)])
def test_concat_alignments(src_mis, dst_mis):
    lens = [1, 0, 15, 16, 17, 31, 33, 1000, 65536, 65537, 3, 200001, 0, 2]
    _check(lens, src_mis, dst_mis, seed=dst_mis)


def test_concat_many_segments_and_large():
    rng = np.random.default_rng(7)
    lens = [int(x) for x in rng.integers(0, 40000, 300)] + [1_150_000, 3_000_001]  # > 96 per launch: several launches
    _check(lens, (0, 9, 4), 3, seed=7)


def test_concat_none():
    assert J.concat_segments(0, 0, [], [], 0) == 0
