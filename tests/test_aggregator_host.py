"""Host-side logic of the processor mirrors (no device): the radix-bucket rule."""
from databend_amd import column as col
from databend_amd.aggregator import HashTableConfig, partial_bucket_bits, payload_tuple_size


def test_radix_bits_rule():
    """maybe_repartition's rule (EAGG/aggregate_hashtable.rs:453-503) on the shared hint."""
    c = HashTableConfig(partial_agg=True)
    ts = payload_tuple_size([col.Int64], 1)
    assert ts == 24
    assert partial_bucket_bits(c, 10_000, ts) == 3           # 240 KB / 8 buckets
    assert partial_bucket_bits(c, 100_000, ts) == 5          # 2.4 MB: 300 KB / 8 > 256 KiB
    assert partial_bucket_bits(c, 10, ts) == 5               # the hint never goes back
    assert partial_bucket_bits(c, 10**8, ts) == 7
    cl = HashTableConfig(partial_agg=True).cluster_with_partial(True, 4)
    assert partial_bucket_bits(cl, 100_000, ts) == 7         # cluster: +4 at a time
    assert payload_tuple_size([col.String, col.Int32.wrap_nullable()], 2) == 1 + 12 + 4 + 8 + 8
