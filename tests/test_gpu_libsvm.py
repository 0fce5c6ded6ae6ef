"""GPU libsvm ingest vs the restated Spark parser (oracle/libsvm_ref.py), and the fused
libsvm -> projection pipeline vs the oracle product."""
import numpy as np
import pytest
import scipy.sparse as sp

from oracle import smmp
from oracle.libsvm_ref import ParseError, parse_text
from randomprojection_amd import Projector, srp_matrix as sm
from randomprojection_amd.libsvm import LibsvmFormatError, parse_bytes, parse_device, project_libsvm, project_text_stream

pytestmark = pytest.mark.gpu


def random_text(rng, n, m, extras=True):
    out = []
    for i in range(n):
        k = int(rng.integers(0, 25))
        idx = np.sort(rng.choice(m, size=k, replace=False)) + 1
        fmt = rng.integers(0, 6, size=k)
        items = []
        for j, f in zip(idx, fmt):
            v = [f"{rng.integers(-9, 10)}", f"{rng.standard_normal():.6g}", f"{rng.random():.3e}",
                 "1", f"{rng.integers(0, 1000)}.{rng.integers(0, 99)}", f".{rng.integers(1, 999)}"][f]
            items.append(f"{j}:{v}")
        sep = "  " if (extras and i % 7 == 0) else " "
        label = ["1", "0", "-1", "+1", "0.5", "3e0"][i % 6]
        line = label + (sep + sep.join(items) if items else "")
        if extras and i % 11 == 0:
            line = "  " + line + " \t"
        out.append(line)
        if extras and i % 13 == 0:
            out.append("# comment line")
        if extras and i % 17 == 0:
            out.append("")
    return ("\n".join(out) + ("\n" if n % 2 else "")).encode()


def same(a, b):
    return a.dtype == b.dtype and np.array_equal(np.asarray(a).view(np.uint8), np.asarray(b).view(np.uint8))


@pytest.mark.parametrize("seed", [0, 1, 2])
def test_parse_matches_oracle(seed):
    rng = np.random.default_rng(seed)
    m = 100_000
    txt = random_text(rng, 3000 + seed * 1000, m)
    lab, ip, ix, vx = parse_text(txt, m)
    labels, X = parse_bytes(txt, m)
    assert same(labels, lab) and np.array_equal(X.indptr, ip) and np.array_equal(X.indices, ix)
    assert same(X.data, vx)


def test_special_literals_and_edges():
    txt = b"1 1:NaN 2:-Infinity 3:+Infinity 4:-0 5:1e21 6:100000000000000000000000 7:0.000001 8:1.\n\n#x\n2\n"
    lab, ip, ix, vx = parse_text(txt, 10)
    labels, X = parse_bytes(txt, 10)
    assert same(labels, lab) and np.array_equal(X.indptr, ip) and np.array_equal(X.indices, ix)
    assert same(X.data, vx)


@pytest.mark.parametrize("line", ["1 0:1", "1 3:1 3:2", "1 101:1", "x 1:1", "1 a:1", "1 3:", "1 3:x", "1\t3:1"])
def test_errors_report_line(line):
    txt = ("2 1:1\n# c\n" + line + "\n1 1:1\n").encode()
    with pytest.raises(ParseError) as ref:
        parse_text(txt, 100)
    with pytest.raises(LibsvmFormatError) as got:
        parse_bytes(txt, 100)
    assert got.value.line == ref.value.line == 2


def test_project_libsvm_end_to_end(tmp_path):
    rng = np.random.default_rng(5)
    m, p = 200_000, 1024
    txt = random_text(rng, 20_000, m, extras=False)
    path = tmp_path / "train.libsvm"
    path.write_bytes(txt)
    R = sm.projection_operand(sm.sparse_random_matrix(p, m, random_state=123))
    P = Projector(R)
    lab, ip, ix, vx = parse_text(txt, m)
    A = sp.csr_matrix((vx, ix, ip), shape=(len(lab), m))
    Cp, Cj, Cx, _, _ = smmp.matmat(A, R)
    Cj_s, Cx_s = smmp.sorted_rows(Cp, Cj, Cx)
    got_ids, got_lab, got_C = [], [], []
    for ids, labels, C in project_libsvm(str(path), P, chunk_bytes=100_000):
        got_ids.append(ids)
        got_lab.append(labels)
        got_C.append(C)
    C = sp.vstack(got_C).tocsr()
    assert same(np.concatenate(got_lab), lab)
    assert np.array_equal(C.indptr, Cp) and np.array_equal(C.indices, Cj_s) and same(C.data, Cx_s)
    assert all(int(i[0]) == (k << 33) for k, i in enumerate(got_ids))


def _tricky_literals(rng):
    """Literals outside Clinger's fast path: 17-digit shortest round trips, 20-40 digit values,
    exact decimal expansions of half-way points between adjacent doubles (ties: round half even)
    and their neighbours 1e-30 relative away (the exact slow path), |exp| > 22, subnormals,
    overflow/underflow, hex literals and Java type suffixes."""
    import decimal

    decimal.getcontext().prec = 1200
    out = []
    for _ in range(300):
        x = float(rng.standard_normal() * 10.0 ** rng.integers(-30, 30))
        out.append(repr(x))
        out.append(f"{x:.25e}")
        out.append(f"{x:.40g}")
    for _ in range(200):  # half-way points and near misses
        x = abs(float(rng.standard_normal() * 10.0 ** rng.integers(-300, 300))) or 1.0
        y = np.nextafter(x, np.inf)
        h = (decimal.Decimal(x) + decimal.Decimal(y)) / 2
        out.append(format(h, "f") if abs(h.adjusted()) < 30 else format(h, "e"))
        for eps in ("1e-60", "-1e-60"):
            v = h * (1 + decimal.Decimal(eps))
            out.append(format(v, "e"))
    for e in range(-330, -300):  # subnormals and the underflow edge
        out.append(f"{rng.integers(1, 99999)}e{e}")
        out.append(f"4.9e{e - 294}" if e == -330 else f"2.4703282292062327e-324")
    out += ["1e400", "-1e400", "1e-400", "2.2250738585072011e-308", "2.2250738585072012e-308",
            "1.7976931348623157e308", "1.7976931348623158e308", "1.7976931348623159e308",
            "0x1.8p1", "-0x.1p-2", "0X1P-1074", "0x1.fffffffffffff8p1023", "0x1.000000000000081p0", "1.5f", "2d",
            "123456789012345678901234567890", "0.1234567890123456789012345678901234567890e-5",
            "9007199254740993", "9007199254740993.0000000000000000001", "1" + "0" * 400 + "e-400"]
    return out


def test_every_java_double_literal_exact():
    """Every value Java's Double.parseDouble accepts, correctly rounded to binary64 (labels) and
    then to float32 (features, the recipe's astype(np.float32)), against the restated parser."""
    rng = np.random.default_rng(17)
    lits = _tricky_literals(rng)
    lines = []
    for k in range(0, len(lits), 5):
        chunk = lits[k:k + 5]
        lines.append(chunk[0] + "".join(f" {i + 1}:{v}" for i, v in enumerate(chunk)))
    txt = ("\n".join(lines) + "\n").encode()
    lab, ip, ix, vx = parse_text(txt, 10)
    labels, X = parse_bytes(txt, 10)
    bad = np.nonzero(labels.view(np.uint64) != lab.view(np.uint64))[0]
    assert bad.size == 0, [(lines[i].split()[0], labels[i], lab[i]) for i in bad[:5]]
    assert np.array_equal(X.indptr, ip) and np.array_equal(X.indices, ix)
    assert same(X.data, vx)


@pytest.mark.parametrize("order", ["sorted", "scipy"])
@pytest.mark.parametrize("chunk", [4096, 100_000, 64 << 20])
def test_project_text_stream_vs_oracle(order, chunk):
    """Boundary 3 in one native call (rp_libsvm_project_stream): chunks of whole lines overlapped
    upload / parse + projection / download; comments, blank lines, odd spacing, a last line without
    its newline, chunks smaller than a line; every row's label, indices and value bits equal the
    restated Spark parser + scipy kernel."""
    rng = np.random.default_rng(23)
    m, p = 200_000, 1024
    txt = random_text(rng, 7001, m) + b"1 5:2.5 77:-1e-3"  # no trailing newline
    R = sm.projection_operand(sm.sparse_random_matrix(p, m, random_state=123))
    P = Projector(R)
    lab, ip, ix, vx = parse_text(txt, m)
    A = sp.csr_matrix((vx, ix, ip), shape=(len(lab), m))
    Cp, Cj, Cx, _, _ = smmp.matmat(A, R)
    if order == "sorted":
        Cj, Cx = smmp.sorted_rows(Cp, Cj, Cx)
    labels, gp, gj, gx = project_text_stream(txt, P, order=order, chunk_bytes=chunk)
    assert same(labels, lab)
    assert np.array_equal(gp, Cp) and np.array_equal(gj, Cj) and same(gx, Cx)


def test_project_text_stream_synthetic_kdd_text():
    """Text written on the GPU from KDD-shaped rows (rp_synth_libsvm_device, 6-17 digit values):
    streamed in 1 MB chunks into preallocated arrays, the result equals parsing the whole text in
    one device call and projecting it with rp_project_device; sampled lines equal the oracle."""
    import torch

    from randomprojection_amd import synth

    m, p, n = 2_000_000, 4096, 150_000
    R = sm.projection_operand(sm.sparse_random_matrix(p, m, random_state=123))
    P = Projector(R)
    Ap, Aj, Ax = synth.kdd_rows_device(n, m, seed=9)
    t, off = synth.libsvm_text_device(Ap, Aj, seed=3)
    text = t.cpu().numpy()
    offs = off.cpu().numpy()
    assert offs[-1] == text.size and text[-1] == 10
    labels, gp, gj, gx = project_text_stream(text, P, order="scipy", chunk_bytes=1 << 20)
    assert labels.size == n
    # the same text parsed whole on the device, then projected device-resident
    dl, dp, dj, dx = parse_device(t, int(t.numel()), m)
    assert torch.equal(dj, Aj)  # the synthetic text carries the generator's columns
    nnz = int(dj.numel())
    cap = int(1.1 * nnz * P.nnz / P.m) + 4096
    Cp = torch.empty(n + 1, dtype=torch.int32, device="cuda")
    Cj = torch.empty(cap, dtype=torch.int32, device="cuda")
    Cx = torch.empty(cap, dtype=torch.float32, device="cuda")
    k = P.project_device(dp, dj, dx, Cp, Cj, Cx, nnz_a=nnz)
    assert same(labels, dl.cpu().numpy())
    assert np.array_equal(gp, Cp.cpu().numpy()) and np.array_equal(gj, Cj[:k].cpu().numpy())
    assert same(gx, Cx[:k].cpu().numpy())
    rows = np.sort(np.random.default_rng(1).choice(n, 500, replace=False))
    sample = b"".join(text[offs[r]:offs[r + 1]].tobytes() for r in rows)
    l_ref, p_ref, j_ref, v_ref = parse_text(sample, m)
    assert same(labels[rows], l_ref)
    W = smmp.matmat(sp.csr_matrix((v_ref, j_ref, p_ref), shape=(rows.size, m)), R)
    G = sp.csr_matrix((gx, gj, gp), shape=(n, p))[rows]
    assert np.array_equal(G.indptr, W[0]) and np.array_equal(G.indices, W[1]) and same(G.data, W[2])


def test_project_text_stream_errors():
    """A malformed line reports its 0-based line number in the whole text (not in its chunk); too
    small preallocated outputs give RP_ERR_CAPACITY."""
    from randomprojection_amd import _native as nat

    m = 1000
    R = sm.projection_operand(sm.sparse_random_matrix(64, m, random_state=1))
    P = Projector(R)
    good = "".join(f"{i % 2} {i % 900 + 1}:1.5 {i % 900 + 50}:2\n" for i in range(5000))
    txt = (good + "1 7:1 3:2\n" + good).encode()
    with pytest.raises(LibsvmFormatError) as e:
        project_text_stream(txt, P, chunk_bytes=4096)
    assert e.value.line == 5000
    small = (np.empty(10), np.empty(11, np.int32), np.empty(100, np.int32), np.empty(100, np.float32))
    with pytest.raises(nat.RPError) as c:
        project_text_stream(good.encode(), P, chunk_bytes=4096, out=small)
    assert c.value.code == nat.RP_ERR_CAPACITY


# ---- the workgroup-cooperative parser (rp_libsvm.hip coop_parse_kernel): texts without tabs or
# comments, so every 8 KB block is parsed one thread per token from LDS (a block holding a tab, a
# '#' token or a window past 12 KB is parsed one thread per line instead)
WHY = {"label is not a number": "label", "feature index is not an int": "index", "item without ':value'": "novalue",
       "feature value is not a number": "value", "indices should be one-based and in ascending order": "order",
       "feature index >= numFeatures": "range"}


def spaced_text(rng, n, m, long_every=0):
    """Lines with single and double separators, leading / trailing spaces, blank and all-space lines,
    label-only lines; with ``long_every``, some lines of thousands of items (windows past 12 KB)."""
    out = []
    for i in range(n):
        k = int(rng.integers(0, 25)) if not (long_every and i % long_every == long_every - 1) else 3000
        idx = np.sort(rng.choice(m, size=k, replace=False)) + 1
        items = [f"{j}:{v}" for j, v in zip(idx, rng.standard_normal(k).astype(np.float32))]
        sep = "  " if i % 5 == 0 else " "
        line = ["1", "0", "-1", "+1", "0.5", "3e0"][i % 6] + (sep + sep.join(items) if items else "")
        if i % 9 == 0:
            line = "   " + line + "  "
        out.append(line)
        if i % 23 == 0:
            out.append("" if i % 2 else "    ")
    return ("\n".join(out) + "\n").encode()


@pytest.mark.parametrize("seed,long_every", [(10, 0), (11, 0), (12, 400)])
def test_coop_parse_matches_oracle(seed, long_every):
    rng = np.random.default_rng(seed)
    m = 50_000
    txt = spaced_text(rng, 6000, m, long_every)
    assert b"\t" not in txt and b"#" not in txt
    lab, ip, ix, vx = parse_text(txt, m)
    labels, X = parse_bytes(txt, m)
    assert same(labels, lab) and np.array_equal(X.indptr, ip) and np.array_equal(X.indices, ix)
    assert same(X.data, vx)


@pytest.mark.parametrize("bad", ["1 0:1", "1 3:1 3:2", "1 101:1", "x 1:1", "1 a:1", "1 3:", "1 3:x", "1 3:1 :2",
                                 "1 3:x 2:1", "1 5:1 4:x", "1 2:1 1:1 200:1", "1 4:1 200:1 3:1", "1 2 3:1",
                                 "y 1:x 0:1", "1 7:1 8:1 9:1 10:zz 5:1"])
@pytest.mark.parametrize("where", [5, 700, 1999])
def test_coop_errors_first_in_line_and_text(bad, where):
    """The first error a sequential parse meets: the smallest line, and in it the leftmost failing
    item, whatever the cooperative parser's thread order (a second bad line comes later)."""
    rng = np.random.default_rng(where)
    lines = spaced_text(rng, 2000, 100).decode().split("\n")[:-1]
    lines[where] = bad
    lines.insert(min(where + 50, len(lines)), "1 1:1 1:2")
    txt = ("\n".join(lines) + "\n").encode()
    with pytest.raises(ParseError) as ref:
        parse_text(txt, 100)
    with pytest.raises(LibsvmFormatError) as got:
        parse_bytes(txt, 100)
    assert got.value.line == ref.value.line == where
    assert WHY[str(got.value).split(": ", 1)[1]] == ref.value.why
