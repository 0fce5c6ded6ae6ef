"""ORACLE — TEST INFRASTRUCTURE ONLY (never imported by the product).

Restatement of Spark's libsvm reader as used by the reference
(``spark.read.format("libsvm").load(path, numFeatures=N)``, code/clustermode/randomProjection.py:71):
``MLUtils.loadLibSVMFile`` line filter (``trim``, skip empty and ``#`` lines) and
``MLUtils.parseLibSVMRecord`` (split on ' ', label ``toDouble``, items ``i:v`` with ``toInt - 1``
and ``toDouble``, strictly ascending 0-based indices), plus ``numFeatures`` bound.
Java's ``Double.parseDouble`` / ``Integer.parseInt`` grammars are restated with regular
expressions (Python's float() accepts more, e.g. "inf", "1_0").

Parity: UNPINNED against Spark itself — Spark/JVM are not in the container and the reference
holds no libsvm fixtures; this restates the published Scala source. The GPU ingest is checked
against this restatement.
"""
from __future__ import annotations

import re

import numpy as np

_JDOUBLE = re.compile(r"^[+-]?(NaN|Infinity|((\d+\.?\d*|\.\d+)([eE][+-]?\d+)?)[fFdD]?)$")
_JHEX = re.compile(r"^[+-]?0[xX]([0-9a-fA-F]+\.?|[0-9a-fA-F]*\.[0-9a-fA-F]+)[pP][+-]?\d+[fFdD]?$")
_JINT = re.compile(r"^[+-]?\d+$")


class ParseError(ValueError):
    def __init__(self, line_no, why):
        super().__init__(f"line {line_no}: {why}")
        self.line = line_no
        self.why = why


def java_trim(s: str) -> str:
    i, j = 0, len(s)
    while i < j and ord(s[i]) <= 32:
        i += 1
    while j > i and ord(s[j - 1]) <= 32:
        j -= 1
    return s[i:j]


def java_double(s: str) -> float:
    s = java_trim(s)
    if _JHEX.match(s):  # HexFloatingPointLiteral (binary exponent required), correctly rounded
        try:
            return float.fromhex(s[:-1] if s[-1] in "fFdD" else s)
        except OverflowError:  # rounds past the largest double: Java gives +-Infinity
            return float("-inf") if s[0] == "-" else float("inf")
    if not _JDOUBLE.match(s):
        raise ValueError(s)
    if s[-1] in "fFdD" and "Infinity" not in s and "NaN" not in s:
        s = s[:-1]
    return float(s.replace("Infinity", "inf"))


def java_int(s: str) -> int:
    if not _JINT.match(s):
        raise ValueError(s)
    v = int(s)
    if not -(2**31) <= v < 2**31:
        raise ValueError(s)
    return v


def java_split(s: str, sep: str):
    """String.split(sep) for a one-character literal separator: trailing empty strings removed."""
    parts = s.split(sep)
    while parts and parts[-1] == "":
        parts.pop()
    return parts


def parse_text(text: bytes, num_features: int):
    """-> (labels float64, indptr int64, indices int32, values float32); raises ParseError."""
    labels, indptr, indices, values = [], [0], [], []
    for line_no, raw in enumerate(text.decode("latin-1").split("\n")):
        line = java_trim(raw)
        if not line or line.startswith("#"):
            continue
        items = java_split(line, " ")
        try:
            label = java_double(items[0])
        except ValueError:
            raise ParseError(line_no, "label") from None
        prev = -1
        for item in (it for it in items[1:] if it):
            parts = java_split(item, ":")
            if len(parts) < 2:
                raise ParseError(line_no, "novalue")
            try:
                idx = java_int(parts[0]) - 1
            except ValueError:
                raise ParseError(line_no, "index") from None
            try:
                val = java_double(parts[1])
            except ValueError:
                raise ParseError(line_no, "value") from None
            if idx <= prev:
                raise ParseError(line_no, "order")
            if idx >= num_features:
                raise ParseError(line_no, "range")
            prev = idx
            indices.append(idx)
            values.append(val)
        labels.append(label)
        indptr.append(len(indices))
    with np.errstate(over="ignore"):
        vals32 = np.array(values, np.float64).astype(np.float32)
    return np.array(labels, np.float64), np.array(indptr, np.int64), np.array(indices, np.int32), vals32
