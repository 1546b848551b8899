"""The bf16 wire kernels of the view-DP exchange (hidegs_amd/csrc/wire.hip) against the torch
definitions they replace in view_dp._Bucket, bit for bit (integer-exact: bf16 bit patterns)."""
import pytest
import torch

from hidegs_amd import wire

pytestmark = pytest.mark.gpu


def _specials(n, seed):
    """Random fp32 over every exponent, with infinities, NaNs, signed zeros, denormals and exact
    rounding ties (low half 0x8000) mixed in."""
    g = torch.Generator(device="cuda").manual_seed(seed)
    bits = torch.randint(-2**31, 2**31, (n,), device="cuda", generator=g, dtype=torch.int64).to(torch.int32)
    x = bits.view(torch.float32).clone()
    x[::97] = float("inf")
    x[1::97] = float("-inf")
    x[2::97] = float("nan")
    x[3::97] = 0.0
    x[4::97] = -0.0
    x[5::97] = 1e-40
    tie = (bits & ~0xFFFF) | 0x8000  # exactly half-way between two bf16 values
    x[6::13] = tie[6::13].view(torch.float32)
    x[7::13] = torch.randn(x[7::13].shape, device="cuda", generator=g)
    return x


def _bits(t):
    return t.view(torch.int16)


@pytest.mark.parametrize("n,pad", [(0, 8), (1, 8), (7, 8), (8, 8), (9, 24), (1000, 1000), (1_000_003, 1_000_016)])
def test_pack_is_to_bfloat16(n, pad):
    x = _specials(n, n)
    dst = torch.full((pad,), 1.0, dtype=torch.bfloat16, device="cuda")
    wire.bf16_pack(x, dst)
    ref = x.to(torch.bfloat16)
    nan = torch.isnan(x)
    assert torch.equal(_bits(dst[:n])[~nan], _bits(ref)[~nan])
    assert bool(torch.isnan(dst[:n].float())[nan].all())
    assert bool((_bits(dst[:n])[nan] == 0x7FC0).all())  # c10's canonical NaN
    assert bool((_bits(dst[n:]) == 0).all())


def test_pack_unaligned_source():
    x = _specials(10_001, 5)
    src = x[1:]  # 4 bytes past a 16-byte boundary: the element-wise path
    dst = torch.empty(10_000, dtype=torch.bfloat16, device="cuda")
    wire.bf16_pack(src, dst)
    ok = ~torch.isnan(src)
    assert torch.equal(_bits(dst)[ok], _bits(src.to(torch.bfloat16))[ok])


@pytest.mark.parametrize("world", [1, 2, 3, 8])
@pytest.mark.parametrize("chunk", [8, 1000, 1003, 262_144])
def test_sum_ranks_is_the_rank_order_fp32_sum(world, chunk):
    g = torch.Generator(device="cuda").manual_seed(world * 1000 + chunk)
    parts = (torch.randn(world, chunk, device="cuda", generator=g) *
             torch.logspace(-3, 3, chunk, device="cuda")).to(torch.bfloat16)
    parts[:, ::101] = torch.tensor(float("inf")).to(torch.bfloat16)
    got = wire.bf16_sum_ranks(parts)
    acc = parts[0].to(torch.float32)
    for r in range(1, world):
        acc += parts[r].to(torch.float32)
    ref = acc.to(torch.bfloat16)
    assert torch.equal(_bits(got), _bits(ref))


@pytest.mark.parametrize("n", [0, 1, 8, 13, 999_999])
def test_unpack_is_float(n):
    h = _specials(n, 3).to(torch.bfloat16)
    src = torch.cat([h, torch.zeros(5, dtype=torch.bfloat16, device="cuda")])  # longer source: front n used
    dst = torch.empty(n, device="cuda")
    wire.bf16_unpack(src, dst)
    assert torch.equal(dst.view(torch.int32), h.float().view(torch.int32))


def test_wire_rejects_wrong_dtypes_and_sizes():
    x = torch.zeros(16, device="cuda")
    with pytest.raises(RuntimeError):
        wire.bf16_pack(x, torch.empty(8, dtype=torch.bfloat16, device="cuda"))
    with pytest.raises(RuntimeError):
        wire.bf16_pack(x, torch.empty(16, dtype=torch.float16, device="cuda"))
    with pytest.raises(RuntimeError):
        wire.bf16_unpack(torch.empty(4, dtype=torch.bfloat16, device="cuda"), x)


@pytest.mark.parametrize("n", [1, 7, 8, 9, 1000, 2_000_003])
@pytest.mark.parametrize("ranks", [1, 3, 8])
def test_mask_pack_and_union_count_match_the_definitions(n, ranks):
    from hidegs_amd.view_dp import pack_mask, unpack_mask
    g = torch.Generator(device="cuda").manual_seed(n + ranks)
    masks = [torch.rand(n, device="cuda", generator=g) < p for p in torch.linspace(0.05, 0.9, ranks).tolist()]
    packed = [wire.mask_pack(m) for m in masks]
    for m, b in zip(masks, packed):
        assert torch.equal(b, pack_mask(m))
    flat = torch.stack(packed)
    union, count = wire.mask_union_count(flat, n)
    ref = unpack_mask(flat, n).sum(0, dtype=torch.int32)
    assert torch.equal(union, ref > 0)
    assert torch.equal(count, ref.to(torch.float32).unsqueeze(1))
