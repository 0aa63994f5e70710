"""The cache layer's compression decision, exported by the library (no GPU needed):
strip_known_cache_key_suffixes (reference src/cache.rs:226-275) and
CacheManager::effective_compression (src/cache.rs:1158-1178) — rule override, size threshold,
then the extension denylist (src/compression.rs:252-308) on the key with its suffixes stripped.

Vectors: the cache-key shapes of the reference's own tests (tests/cache_key_length_test.rs:143-146,
tests/cache_cleanup_new_format_test.rs:50-52) and the grammar of generate_part_cache_key /
generate_range_cache_key described at cache.rs:200-225."""
import pytest

import s3hc_lz4 as S

STRIP = [
    ("bucket/object.jpg:range:0-8388607", "bucket/object.jpg"),
    ("my-bucket/object.jpg:version:abc123:range:0-8388607", "my-bucket/object.jpg:version:abc123"),
    ("bucket/big.zip:part:3", "bucket/big.zip"),
    ("bucket/big.zip:part:3:range:0-1048575", "bucket/big.zip"),
    ("bucket/plain.json", "bucket/plain.json"),
    ("bucket/a:b:c.jpg", "bucket/a:b:c.jpg"),                     # colons inside the object key stay
    ("k:range:abc", "k:range:abc"),                               # body not <digits>-<digits>
    ("k:range:5-", "k:range:5-"),
    ("k:range:-5", "k:range:-5"),
    ("k:range:1-2-3", "k:range:1-2-3"),                           # split at the first '-': "2-3" not digits
    ("k:range:0:99", "k:range:0:99"),                             # the RAM-cache grammar is not stripped (cache.rs:214-224)
    ("k:part:", "k:part:"),
    ("k:part:12a", "k:part:12a"),
    ("k:range:0-9:part:3", "k:range:0-9"),                         # range is not last: only the part is stripped
    ("k:part:1:part:2", "k:part:1"),                               # one part suffix only
    ("", ""),
    ("photos/été.png:range:1-2", "photos/été.png"),  # multi-byte UTF-8 key
]


@pytest.mark.parametrize("key,want", STRIP)
def test_strip_known_cache_key_suffixes(key, want):
    assert S.strip_known_cache_key_suffixes(key) == want


R = S.ResolvedSettings
DECIDE = [
    # (enabled, from_rule, threshold, key, size) -> compress?
    ((True, False, 1024, "bucket/log.json:range:0-65535", 65536), True),
    ((True, False, 1024, "bucket/img.jpg:range:0-65535", 65536), False),    # denylisted after stripping
    ((True, False, 1024, "bucket/IMG.JPEG:part:2", 65536), False),           # case-insensitive extension
    ((True, False, 1024, "bucket/archive.tar.gz", 65536), False),
    ((True, False, 1024, "bucket/img.jpg:range:0:99", 65536), True),        # RAM grammar: ext "jpg:range:0:99"
    ((True, True, 1024, "bucket/img.jpg:range:0-65535", 65536), True),      # a rule wins over the denylist
    ((True, True, 1024, "bucket/img.jpg", 1023), False),                    # ... but not over the threshold
    ((True, False, 1024, "bucket/log.json", 1024), True),                   # size == threshold passes
    ((True, False, 1024, "bucket/log.json", 1023), False),
    ((False, True, 0, "bucket/log.json", 1 << 30), False),                 # disabled wins over everything
    ((True, False, 0, "bucket/dir.with.dot/file", 0), True),               # no extension in the last segment
    ((True, False, 0, "bucket/file.", 10), True),                          # empty extension
]


@pytest.mark.parametrize("args,want", DECIDE)
def test_effective_compression(args, want):
    en, rule, thr, key, size = args
    assert S.effective_compression(R(en, rule), thr, key, size) is want


def test_handler_uses_its_threshold():
    h = S.CompressionHandler.__new__(S.CompressionHandler)
    h.engine = None
    h.h = S.lib.s3hc_handler_new(None, 4096, 1)  # the decision never touches the device
    try:
        assert h.effective_compression(R(True, False), "b/x.json", 4096) is True
        assert h.effective_compression(R(True, False), "b/x.json", 4095) is False
        assert h.effective_compression(R(True, False), "b/x.png:range:0-1", 1 << 20) is False
    finally:
        S.lib.s3hc_handler_free(h.h)
        h.h = None


def test_config3_routing_by_cache_key():
    """Config 3's mixed corpus routed the way the reference routes it: JPEG ranges arrive with
    ':range:' cache keys and go to store-mode; JSON ranges are compressed."""
    keys = [f"media-assets/blob-{i:05d}{'.json' if i % 2 == 0 else '.jpg'}:range:{i * 65536}-{i * 65536 + 65535}"
            for i in range(64)]
    modes = [0 if S.effective_compression(R(), 1024, k, 65536) else 1 for k in keys]
    assert modes == [i % 2 for i in range(64)]
