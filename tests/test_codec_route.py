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
    # a whole 16-core host outruns one GPU's queue (37-44 GiB/s measured) at any load,
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
    """profiles/r06/queue_split.jsonl (RS(8+4) 1 MiB encode + sums, pinned, one device,
    the product build): 3.11 / 23.6 / 35.6 / 38.4 GiB/s at 1 / 16 / 64 / 256 submitters."""
    meas = {1: 3.11, 16: 23.57, 64: 35.57, 256: 38.44}
    for t, g in meas.items():
        got = e.device_codec_Bps("encode", t, MiB) / 2**30
        assert abs(got - g) / g < 0.08, (t, got, g)
