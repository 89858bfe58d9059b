"""CPU test of the digest routing rule (zs3server_amd/etag.py digest_on_device, VERDICT
r04 item 8): single parts and small batches hash on the host (internal/etag/reader.go:114,
internal/hash/reader.go:137); only many concurrent parts go to zs3_md5_parts /
zs3_sha256_parts, the threshold following from the device's per-message chain roof
 against the host's per-core rate."""
from zs3server_amd import etag as E

MiB = 1 << 20


def test_single_part_stays_on_host():
    for algo in ("md5", "sha256"):
        for size in (1, 64, 5 * MiB, 5 << 30):
            assert not E.digest_on_device(algo, 1, size, cpu_threads=1, cpu_Bps=1e8)


def test_few_parts_stay_on_host():
    # 4 parts of 5 MiB, 16 cores at 700 MB/s: one core per part is faster than one lane per part
    assert not E.digest_on_device("md5", 4, 5 * MiB, cpu_threads=16, cpu_Bps=7e8)
    assert not E.digest_on_device("sha256", 64, 5 * MiB, cpu_threads=16, cpu_Bps=4e8)


def test_many_concurrent_parts_go_to_the_device():
    # 256 parts of 5 MiB (the multipart-upload case of DESIGN.md §12.5) on 16 host cores
    assert E.digest_on_device("md5", 256, 5 * MiB, cpu_threads=16, cpu_Bps=7e8)
    assert E.digest_on_device("md5", 256, 5 * MiB, cpu_threads=16, cpu_Bps=7e8, resident=True)
    assert E.digest_on_device("sha256", 1024, 5 * MiB, cpu_threads=16, cpu_Bps=4e8)


def test_threshold_is_monotone_in_parts_and_cores():
    def first_n(algo, threads, rate):
        for n in range(1, 5000):
            if E.digest_on_device(algo, n, 5 * MiB, threads, rate):
                return n
        return None
    a, b = first_n("md5", 16, 7e8), first_n("md5", 32, 7e8)
    assert a is not None and b is not None and b > a
    # once the device wins it keeps winning up to the lane count
    assert all(E.digest_on_device("md5", n, 5 * MiB, 16, 7e8) for n in range(a, E.GPU_DIGEST_LANES, 97))


def test_host_rate_calibration_runs():
    assert E.host_digest_Bps("md5", 1 << 20) > 1e6
