"""examples/compression_demo.py (counterpart of the reference's examples/compression_demo.rs,
BASELINE.json configs[0]) runs end to end on the GPU with the reference demo's decisions."""
import os
import sys

import pytest

pytestmark = pytest.mark.gpu
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "examples"))


def test_compression_demo_decisions(engine):
    import compression_demo as D

    lines = []
    results, st = D.demo(engine, out=lines.append)
    deny = {f for f, d, s, r in results if d}
    assert deny == {"photo.jpg", "video.mp4", "archive.zip", "document.pdf", "music.mp3"}
    for f, d, should, r in results:
        assert should == (not d) and r.was_compressed == should
        assert r.algorithm == 0  # both paths are tagged Lz4 (compression.rs:376-460)
        assert (r.compressed_size < r.original_size) == should
    assert st.total_objects_compressed == 5 and st.total_objects_uncompressed == 5
    assert st.compression_failures == 0 and st.decompression_failures == 0
    assert "Content-Aware Compression Demo" in lines[0]


def test_config1_round_trip(engine):
    import compression_demo as D

    r = D.config1(engine, cpu=True, reps=2)
    assert r["bd"] == "0x70" and r["frame_bytes"] < r["bytes"] // 2
