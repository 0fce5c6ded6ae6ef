"""The libsvm oracle (restated Spark MLUtils.parseLibSVMRecord) on hand-checked cases, and the host
chunker. Parity with Spark itself is unpinned (no JVM/Spark in the container)."""
import numpy as np
import pytest

from oracle.libsvm_ref import ParseError, parse_text
from randomprojection_amd.libsvm import iter_chunks, partition_ids


def test_basic_and_filters():
    txt = b"1 3:1 10:2.5\n# comment\n\n   \n0  1:1   2:-3e2 \n-1\n+1 4:NaN 5:-Infinity 6:1.0d\n"
    lab, ip, ix, vx = parse_text(txt, 100)
    assert list(lab[:3]) == [1.0, 0.0, -1.0] and lab[3] == 1.0
    assert list(ip) == [0, 2, 4, 4, 7]
    assert list(ix) == [2, 9, 0, 1, 3, 4, 5]
    assert vx[0] == 1 and vx[1] == 2.5 and vx[3] == -300 and np.isnan(vx[4]) and vx[5] == -np.inf and vx[6] == 1.0


@pytest.mark.parametrize("line,why", [
    ("1 0:1", "order"), ("1 3:1 3:2", "order"), ("1 5:1 2:1", "order"), ("1 101:1", "range"),
    ("x 1:1", "label"), ("1 a:1", "index"), ("1 3:", "novalue"), ("1 3", "novalue"), ("1 3:x", "value"),
    ("1 :3", "index"), ("1\t3:1", "label"), ("1 3:1e", "value"), ("1 99999999999:1", "index"),
])
def test_errors(line, why):
    with pytest.raises(ParseError) as e:
        parse_text(("2 1:1\n" + line + "\n").encode(), 100)
    assert e.value.line == 1 and e.value.why == why


def test_extra_colon_parts_ignored():
    lab, ip, ix, vx = parse_text(b"1 3:2:9 4:1:\n", 10)
    assert list(ix) == [2, 3] and list(vx) == [2.0, 1.0]


def test_float32_rounding_of_double():
    lab, ip, ix, vx = parse_text(b"1 1:0.1 2:16777217 3:3.4028235677973366e38\n", 10)
    assert vx.dtype == np.float32 and vx[0] == np.float32(0.1) and vx[1] == np.float32(16777216.0)


def test_chunker_aligns_on_newlines(tmp_path):
    lines = [f"{i % 2} {i + 1}:1 {i + 5}:2" for i in range(1000)]
    p = tmp_path / "x.libsvm"
    p.write_text("\n".join(lines))          # no trailing newline
    chunks = list(iter_chunks(str(p), chunk_bytes=777))
    assert b"".join(chunks) == p.read_bytes()
    assert all(c.endswith(b"\n") for c in chunks[:-1])
    long = tmp_path / "long.libsvm"
    long.write_text("1 " + " ".join(f"{i}:1" for i in range(1, 500)) + "\n0 1:1\n")
    assert [c.count(b"\n") for c in iter_chunks(str(long), chunk_bytes=64)] == [1, 1]


def test_partition_ids():
    ids = partition_ids(3, 4)
    assert list(ids) == [(3 << 33) + i for i in range(4)]


def test_java_hex_and_suffix_literals():
    from oracle.libsvm_ref import java_double

    assert java_double("0x1.8p1") == 3.0 and java_double("-0x.1p-2f") == -0.015625
    assert java_double("0X1P-1074") == 5e-324 and java_double("0x1.fffffffffffff8p1023") == float("inf")
    assert java_double("1.5d") == 1.5 and java_double("1e400") == float("inf") and java_double("1e-400") == 0.0
    for bad in ("0x1.8", "0x", "1.5g", "0x1p", "inf", "1_0"):
        with pytest.raises(ValueError):
            java_double(bad)
