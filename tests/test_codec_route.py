"""CPU tests of the per-block routing rule (zs3server_amd/erasure.py codec_on_device,
VERDICT r05 item 3): where the rocm build runs one EncodeData / DecodeDataBlocks /
DecodeDataAndParityBlocks — the batching queue or the reference's own per-goroutine
klauspost path (cmd/erasure-encode.go:83-111, cmd/erasure-decode.go:230-276)."""
import pytest

from zs3server_amd import erasure as e

MiB = 1 << 20
OPS = ("encode", "get", "heal")


@pytest.mark.parametrize("op", OPS)
def test_lone_request_stays_on_host(op):
    for cores in (1, 2, 4, 16, 64):
        assert not e.codec_on_device(op, 1, MiB, cores)


@pytest.mark.parametrize("op", OPS)
def test_many_requests_go_to_device_when_host_cores_are_few(op):
    assert e.codec_on_device(op, 256, MiB, 2)
    assert e.codec_on_device(op, 1024, MiB, 1)
    # a whole 16-core host outruns one GPU's queue (30-43 GiB/s measured) at any load,
    # eight GPUs take over from a few dozen requests
    assert not e.codec_on_device(op, 4096, MiB, 16)
    assert e.codec_on_device(op, 4096, MiB, 16, devices=8)


@pytest.mark.parametrize("op", OPS)
@pytest.mark.parametrize("cores", [1, 2, 3, 4])
def test_threshold_is_monotone(op, cores):
    t = e.codec_device_threshold(op, MiB, cores, max_live=4096)
    assert t is not None and t > 1
    # below the threshold: host; at and above it (checked to 8x): device
    assert not any(e.codec_on_device(op, x, MiB, cores) for x in range(1, t))
    assert all(e.codec_on_device(op, x, MiB, cores) for x in range(t, 8 * t))
    # more host cores never lower the threshold, more devices never raise it
    t_more = e.codec_device_threshold(op, MiB, cores + 1, max_live=4096)
    assert t_more is None or t_more >= t
    assert e.codec_device_threshold(op, MiB, cores, devices=2, max_live=4096) <= t


def test_model_follows_the_measured_queue_curve():
    """profiles/r06/queue_product.jsonl, queue_product2.jsonl (RS(8+4) 1 MiB encode +
    sums, pinned, one device, the product build): 3.16 / 22.3 / 40.3-40.5 GiB/s at 1 / 16 /
    64 submitters.  At 256 the box's 16-core share runs the 256 submitter threads and the
    rate spreads over 31-41 GiB/s between repeats (best 44.2, queue_split_slots.jsonl): the
    model must not promise more than that.  Two parameters (lone-block time, ceiling)
    cannot follow both ends: it is within 8 % at 1 and 16 and 13 % low at 64, on the side
    that keeps blocks on the host."""
    meas = {1: (3.16, 0.08), 16: (22.32, 0.08), 64: (40.4, 0.15)}
    for t, (g, tol) in meas.items():
        got = e.device_codec_Bps("encode", t, MiB) / 2**30
        assert abs(got - g) / g < tol, (t, got, g)
    assert e.device_codec_Bps("encode", 64, MiB) / 2**30 < 40.4
    assert e.device_codec_Bps("encode", 256, MiB) / 2**30 < 1.1 * 44.2
