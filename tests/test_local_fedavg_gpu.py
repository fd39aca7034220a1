"""csrc/comm.hip gfk_local_fedavg: the in-process fold of N client buffers, bit for bit the
group-wise left fold of the eager sequence (parallel/aggregator.py local_fedavg), for the
register path (N <= 8: every client's float4 loaded before the first add) and the
dependent-load path (N > 8), with uneven groups and a range that ends inside a float4."""
import pytest
import torch

from gfedntm_amd.parallel.aggregator import (LOCAL_ALL, LOCAL_BCAST, LOCAL_FIRST,
                                             local_fedavg, prepare_local_fedavg)

pytestmark = pytest.mark.gpu


def _oracle(bufs, groups, off, n):
    tot, j = None, 0
    for g in groups:
        s = bufs[j][off:off + n].clone()
        for k in range(j + 1, j + g):
            s = s + bufs[k][off:off + n]
        j += g
        tot = s if tot is None else tot + s
    return tot


@pytest.mark.parametrize("groups", [[1], [8], [3, 1, 4], [1, 1, 1, 1, 1, 1, 1, 1], [2, 5],
                                    [4, 6], [10]])
@pytest.mark.parametrize("off,n", [(0, None), (8, 1003)])
def test_local_fedavg_matches_left_fold(groups, off, n):
    torch.manual_seed(0)
    total = 4099
    N = sum(groups)
    bufs = [torch.randn(total, device="cuda") * (1 + i) for i in range(N)]
    nn = total - off if n is None else n
    want = _oracle(bufs, groups, off, nn)
    before = [b.clone() for b in bufs]
    prepare_local_fedavg(bufs, groups)
    local_fedavg(bufs, LOCAL_ALL, groups=groups, off=off, n=n)
    torch.cuda.synchronize()
    for b, b0 in zip(bufs, before):
        assert torch.equal(b[off:off + nn], want)
        assert torch.equal(b[:off], b0[:off]) and torch.equal(b[off + nn:], b0[off + nn:])


def test_local_fedavg_first_and_bcast():
    torch.manual_seed(1)
    bufs = [torch.randn(1000, device="cuda") for _ in range(5)]
    want = _oracle(bufs, [5], 0, 1000)
    others = [b.clone() for b in bufs[1:]]
    prepare_local_fedavg(bufs)
    local_fedavg(bufs, LOCAL_FIRST)
    torch.cuda.synchronize()
    assert torch.equal(bufs[0], want)
    assert all(torch.equal(b, o) for b, o in zip(bufs[1:], others))
    local_fedavg(bufs, LOCAL_BCAST)
    torch.cuda.synchronize()
    assert all(torch.equal(b, want) for b in bufs)
