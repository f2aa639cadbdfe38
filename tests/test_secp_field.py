"""secp256k1_host.hpp's field and point arithmetic (the ECIES / BIP-340 host
code) against Python integers and oracle/host_oracle.py's curve code.

The field is five 52-bit limbs reduced lazily (magnitudes tracked by hand in
the point formulas), so these cases aim at the reduction edges: operands at
and above p (fe_from_be takes any 256-bit value), 0, 1, p - 1, all-ones limbs,
and the largest magnitudes the complete formulas feed fe_mul / fe_sub.
CPU-only: tools/secp_field_check.cpp is compiled with g++ here.
"""
import random
import shutil
import subprocess
from pathlib import Path

import pytest

from oracle import host_oracle as H

ROOT = Path(__file__).resolve().parent.parent
P, N = H.P, H.N


@pytest.fixture(scope="module")
def drv(tmp_path_factory):
    if not shutil.which("g++"):
        pytest.skip("g++ not available")
    exe = tmp_path_factory.mktemp("secp") / "sfc"
    subprocess.run(["g++", "-O2", "-std=c++17", str(ROOT / "tools/secp_field_check.cpp"), "-o", str(exe)],
                   check=True)
    return exe


def _run(exe, lines):
    out = subprocess.run([str(exe)], input="\n".join(lines) + "\n", capture_output=True, text=True, check=True)
    return [ln.split() for ln in out.stdout.splitlines()]


def _edge_values():
    m52 = (1 << 52) - 1
    vals = [0, 1, 2, 977, P - 1, P - 2, P, P + 1, (1 << 256) - 1, (1 << 256) - 2, P - (1 << 52), 1 << 255,
            (1 << 208) - 1, m52, m52 << 52, m52 << 104, m52 << 156, ((1 << 48) - 1) << 208, 0x1000003D1,
            P - 0x1000003D1, (1 << 256) - 0x1000003D1]
    rng = random.Random(7)
    vals += [rng.getrandbits(256) for _ in range(40)]
    return vals


def test_field_ops_match_python(drv):
    vals = _edge_values()
    rng = random.Random(11)
    pairs = [(a, b) for a in vals[:21] for b in vals[:21]] + [(rng.choice(vals), rng.choice(vals)) for _ in range(300)]
    res = _run(drv, ["F %064x %064x" % (a, b) for a, b in pairs])
    for (a, b), r in zip(pairs, res):
        got = [int(x, 16) for x in r]
        want = [a * b % P, a * a % P, (a + b) % P, (a - b) % P, 21 * a % P]
        if a % P:
            want.append(pow(a, P - 2, P))
        assert got == want, (hex(a), hex(b))


def test_field_largest_magnitudes(drv):
    """(8a)(4b) - 8a and (8a)^2 with the sums left unreduced, as in pt_dbl's z3
    chain (magnitude 8 into fe_mul) and fe_sub's 16p bound."""
    vals = _edge_values()
    pairs = [(a, b) for a in vals[:12] for b in vals[:12]] + list(zip(vals[21:], reversed(vals[21:])))
    res = _run(drv, ["C %064x %064x" % (a, b) for a, b in pairs])
    for (a, b), r in zip(pairs, res):
        a8, b4 = 8 * a, 4 * b
        assert [int(x, 16) for x in r] == [(a8 * b4 - a8) % P, a8 * a8 % P], (hex(a), hex(b))


def _ser(pt):
    return "inf" if pt is None else H.ser_uncompressed(pt).hex()


def test_point_mul_matches_oracle(drv):
    rng = random.Random(3)
    ks = [1, 2, 3, 15, 16, 17, N - 1, N - 2, (N - 1) // 2, 1 << 128, (1 << 128) - 1, 1 << 255] + \
         [rng.randrange(1, N) for _ in range(12)]
    q = H.point_mul(0xC0FFEE)
    lines = ["G %064x" % k for k in ks] + ["P %064x %064x %064x" % (k, q[0], q[1]) for k in ks]
    res = _run(drv, lines)
    for k, r in zip(ks, res[:len(ks)]):
        assert r == [_ser(H.point_mul(k))], hex(k)
    for k, r in zip(ks, res[len(ks):]):
        assert r == [_ser(H.point_mul(k, q))], hex(k)
