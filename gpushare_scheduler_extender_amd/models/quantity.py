"""Kubernetes resource.Quantity parsing (pure Python, exact).

``Quantity.Value()`` rounds up to an integer
(``vendor/k8s.io/apimachinery/pkg/api/resource/quantity.go:693-695``); the
reference sums container limits with it (``pkg/utils/pod.go:146-155``).  The
native engine has its own C++ implementation (native/engine/quantity.cc); this
one serves the Python-side tools and cross-checks the engine in tests.
"""
from __future__ import annotations

import math
import re
from fractions import Fraction

_BIN = {"Ki": 10, "Mi": 20, "Gi": 30, "Ti": 40, "Pi": 50, "Ei": 60}
_DEC = {"n": -9, "u": -6, "m": -3, "": 0, "k": 3, "M": 6, "G": 9, "T": 12, "P": 15, "E": 18}
_RE = re.compile(r"^([+-]?)([0-9]+\.?[0-9]*|\.[0-9]+)(.*)$", re.S)  # ASCII digits only, like Go's parser
_INT64_MAX = 2**63 - 1
_INT64_MIN = -(2**63)


def parse_quantity(s) -> int:
    """Return ceil(value) of a quantity string/number, saturated to int64."""
    if isinstance(s, bool):
        raise ValueError(f"invalid quantity {s!r}")
    if isinstance(s, int):
        return max(_INT64_MIN, min(_INT64_MAX, s))
    if isinstance(s, float):
        s = repr(s)
    if isinstance(s, str) and s.isdigit() and s.isascii():  # fast path: plain integers ("64")
        return min(_INT64_MAX, int(s))
    m = _RE.match(str(s))
    if not m:
        raise ValueError(f"quantities must match the regular expression: {s!r}")
    sign, num, suf = m.groups()
    val = Fraction(num)
    if suf in _BIN:
        val *= 2 ** _BIN[suf]
    elif suf in _DEC:
        val *= Fraction(10) ** _DEC[suf]
    elif suf[:1] in ("e", "E") and re.fullmatch(r"[+-]?[0-9]+", suf[1:]):
        val *= Fraction(10) ** int(suf[1:])
    else:
        raise ValueError(f"unknown quantity suffix in {s!r}")
    if sign == "-":
        val = -val
    v = math.ceil(val)
    return max(_INT64_MIN, min(_INT64_MAX, v))


def format_quantity(v: int) -> str:
    return str(int(v))
