"""Go strconv semantics the reference applies to pod labels and annotations.

The drop-in Go plugin parses labels with Go's own strconv (it can call the reference's
filter.StrToUint64 etc. directly); this module is the Python host's faithful copy, used to
pack pods from k8s-style objects and by the tests.

  strToUint / StrToUint64   filter.go:60-74   Atoi; error -> 0; negative wraps to uint64
  GetPodPriority            sort.go:12-18     Atoi value even on error (range -> ±MaxInt64)
  ParseFloat(s, 32)         algorithm.go:103  nearest float32 (as float64); error values:
                                              syntax -> 0, range -> ±Inf
Go version: the reference's go.mod says go 1.15; strconv's Atoi/ParseInt/ParseFloat rules
used here are unchanged since Go 1.13 (underscore handling) — parity unpinned for exotic
strings (no reference execution is possible here).
"""
from __future__ import annotations

import math
import re
from fractions import Fraction
from typing import Tuple

U64 = (1 << 64) - 1
I64_MAX = (1 << 63) - 1
I64_MIN = -(1 << 63)


def atoi(s: str) -> Tuple[int, bool]:
    """strconv.Atoi on a 64-bit platform: (value, ok).  On a syntax error the value is 0;
    on a range error it is clamped to MaxInt64 / MinInt64 (ParseInt's behaviour).

    The range is decided from the digit count before any int() conversion: a label of
    thousands of digits must clamp like Go does, not hit CPython's int-string limit."""
    if 0 < len(s) < 19:  # fast path: no underscores, plain decimal
        body = s[1:] if s[0] in "+-" else s
        if not body or any(not ("0" <= ch <= "9") for ch in body):
            return 0, False
        n = int(body)
        return (-n if s[0] == "-" else n), True
    # ParseInt(s, 10, 0): base 10 (not 0) => underscores are a syntax error
    if not s:
        return 0, False
    neg = s[0] == "-"
    body = s[1:] if s[0] in "+-" else s
    if not body or any(not ("0" <= ch <= "9") for ch in body):
        return 0, False
    digits = body.lstrip("0")
    # 2^63 has 19 digits: anything longer is out of range whatever the digits are
    n = int(digits) if 0 < len(digits) <= 19 else (0 if not digits else 1 << 64)
    if not neg and n > I64_MAX:
        return I64_MAX, False
    if neg and n > (1 << 63):
        return I64_MIN, False
    return (-n if neg else n), True


def str_to_uint(s: str) -> int:
    """filter.strToUint / StrToUint64 (filter.go:60-74): Atoi, error -> 0, uint64 wrap."""
    v, ok = atoi(s)
    return (v & U64) if ok else 0


def pod_priority(s: str) -> int:
    """sort.GetPodPriority (sort.go:12-18): `pri, _ := strconv.Atoi(p)`."""
    return atoi(s)[0]


# ---- ParseFloat -------------------------------------------------------------------------
_DEC = re.compile(r"^([0-9_]*)(?:\.([0-9_]*))?(?:[eE]([+-]?[0-9_]+))?$")
_HEX = re.compile(r"^0[xX]([0-9a-fA-F_]*)(?:\.([0-9a-fA-F_]*))?[pP]([+-]?[0-9_]+)$")


def _underscore_ok(s: str) -> bool:
    """strconv.underscoreOK: '_' only between digits (or after a base prefix)."""
    if s and s[0] in "+-":
        s = s[1:]
    saw = "^"
    i = 0
    hexa = False
    if len(s) >= 2 and s[0] == "0" and s[1].lower() in "box":
        i, saw, hexa = 2, "0", s[1].lower() == "x"
    while i < len(s):
        ch = s[i]
        if ch.isdigit() or (hexa and ch.lower() in "abcdef"):
            saw = "0"
        elif ch == "_":
            if saw != "0":
                return False
            saw = "_"
        else:
            if saw == "_":
                return False
            saw = "!"
        i += 1
    return saw != "_"


def _round_to_bits(q: Fraction, mant_bits: int, emin: int, emax: int) -> float:
    """Correctly round a non-negative rational to an IEEE binary format (RN-even).
    Returns math.inf on overflow."""
    if q == 0:
        return 0.0
    e = q.numerator.bit_length() - q.denominator.bit_length()
    if Fraction(2) ** e > q:
        e -= 1
    e = max(e, emin)                       # subnormals share the minimum exponent
    scale = Fraction(2) ** (e - (mant_bits - 1))
    m = q / scale
    n = m.numerator // m.denominator
    rem = m - n
    if rem > Fraction(1, 2) or (rem == Fraction(1, 2) and n % 2 == 1):
        n += 1
    if n >= (1 << mant_bits):              # mantissa overflow after rounding
        n >>= 1
        e += 1
        scale *= 2
    if e > emax:
        return math.inf
    return float(Fraction(n) * scale)


# Decimal digits that decide a correctly rounded binary64 (767 suffice; Go's decimal
# fallback keeps 800): longer mantissas are cut there with a sticky digit.
_MAX_SIG_DIGITS = 800


def _digits_to_int(d: str, base: int = 10) -> int:
    """int(d, base) without CPython's limit on decimal string length (chunked)."""
    if base != 10 or len(d) <= 4000:
        return int(d, base) if d else 0
    n = 0
    for i in range(0, len(d), 4000):
        c = d[i:i + 4000]
        n = n * 10 ** len(c) + int(c)
    return n


def _exponent(e: str) -> int:
    """Decimal exponent text -> int, saturated (Go saturates the exponent at 10000 too)."""
    e = e.replace("_", "")
    sign = -1 if e.startswith("-") else 1
    body = e.lstrip("+-").lstrip("0") or "0"
    return sign * (int(body) if len(body) <= 9 else 10 ** 9)


def _dec_fraction(ip: str, fp: str, ex: int, bit_size: int):
    """Exact (or sticky-truncated) rational value of ip.fp e ex, or 'inf' / 'zero' when the
    decimal exponent alone decides overflow / underflow (no huge powers are built)."""
    digits = (ip + fp).lstrip("0")
    if not digits:
        return Fraction(0)
    # value = 0.digits * 10^(e10)
    e10 = len(ip + fp) - len(fp) + ex - ((len(ip + fp)) - len(digits))
    hi = 40 if bit_size == 32 else 310    # 0.d * 10^40 > MaxFloat32, 10^310 > MaxFloat64
    lo = -50 if bit_size == 32 else -330  # below half the smallest subnormal
    if e10 > hi:
        return "inf"
    if e10 < lo:
        return "zero"
    if len(digits) > _MAX_SIG_DIGITS:
        sticky = digits[_MAX_SIG_DIGITS:].strip("0") != ""
        digits = digits[:_MAX_SIG_DIGITS] + ("1" if sticky else "")
    return Fraction(_digits_to_int(digits)) * Fraction(10) ** (e10 - len(digits))


def parse_float(s: str, bit_size: int = 64) -> Tuple[float, bool]:
    """strconv.ParseFloat(s, bitSize): (value, ok).  bitSize 32 returns the nearest float32
    as a float64.  Syntax error -> (0, False); overflow -> (±Inf, False); underflow -> ±0.
    The cost is bounded by the string length: huge exponents are decided before any big
    power is built (a '1e999999999' annotation must not stall the packer)."""
    t = s
    neg = False
    if t and t[0] in "+-":
        neg = t[0] == "-"
        t = t[1:]
    low = t.lower()
    if low in ("inf", "infinity"):
        return (-math.inf if neg else math.inf), True
    if low == "nan" and not (s and s[0] in "+-"):
        return math.nan, True
    q = None
    m = _HEX.match(t)
    if m and ("_" not in t or _underscore_ok(s)):
        ip, fp, ex = (m.group(1) or "").replace("_", ""), (m.group(2) or "").replace("_", ""), \
            _exponent(m.group(3))
        if ip or fp:
            mant = _digits_to_int(ip + fp, 16)
            if mant == 0:
                q = Fraction(0)
            else:
                e2 = ex - 4 * len(fp) + mant.bit_length()  # value in [2^(e2-1), 2^e2)
                if e2 > 1100:
                    q = "inf"
                elif e2 < -1200:
                    q = "zero"
                else:
                    q = Fraction(mant) * Fraction(2) ** (ex - 4 * len(fp))
    else:
        m = _DEC.match(t)
        if m and (m.group(1) or m.group(2)):
            if "_" in t and not _underscore_ok(s):
                return 0.0, False
            ip = (m.group(1) or "").replace("_", "")
            fp = (m.group(2) or "").replace("_", "")
            if m.group(3) is not None and not m.group(3).replace("_", "").lstrip("+-"):
                return 0.0, False
            ex = _exponent(m.group(3)) if m.group(3) else 0
            if ip or fp:
                q = _dec_fraction(ip, fp, ex, bit_size)
    if q is None:
        return 0.0, False
    if q == "inf":
        return (-math.inf if neg else math.inf), False
    if q == "zero":
        return (-0.0 if neg else 0.0), True
    if bit_size == 32:
        v = _round_to_bits(q, 24, -126, 127)
    else:
        v = _round_to_bits(q, 53, -1022, 1023)
    if math.isinf(v):
        return (-math.inf if neg else math.inf), False
    return (-v if neg else v), True
