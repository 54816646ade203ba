"""Byte-exact text outputs, CPU only: cpg_format_islands (:287-288) and
cpg_format_model (:207-224) against the oracle's independent restatements (C printf-loop
shortest digits for %f; Python repr for Double.toString) and the committed golden text.
PARITY UNPINNED: Java's Formatter / Double.toString are restated (JDK 19+ shortest digits),
no JVM is available here."""
import os

import numpy as np
import pytest

from oracle import coracle as co
from oracle import pyref as pr

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_islands_text_matches_golden_and_oracle():
    from cpgisland_amd.hmm import format_islands
    g = np.load(os.path.join(ROOT, "tests", "golden", "golden.npz"))
    assert format_islands(g["islands"]).decode() == str(g["islands_txt"])


TRICKY = [0.5, 0.5000005, 0.5000004999999999, 0.1234565, 2.675, 0.9999995, 0.99999949,
          0.6000005, 1.0, 1.23456789e-7, 5e-7, 4.9999999e-7, 123456.9999995, 7.0000005,
          0.3333333333333333, 2.0 / 3.0, 1.0 / 7.0, 0.6, 0.61, 1e-300, 1234567.0000004,
          99.9999995, 0.0, 3.0000000000000004]


@pytest.mark.parametrize("x", TRICKY)
def test_java_f6_tricky_values(x):
    from cpgisland_amd.hmm import format_islands
    rec = np.zeros(1, co.ISLAND_DTYPE)
    rec[0] = (7, 9, 3, 0, x, x)
    txt = format_islands(rec).decode()
    assert txt == co.format_island(rec[0])
    assert txt == "7 9 3 %s %s\n" % (pr.java_f6(x), pr.java_f6(x))


def test_java_f6_random_values():
    from cpgisland_amd.hmm import format_islands
    rng = np.random.default_rng(3)
    recs = np.zeros(2000, co.ISLAND_DTYPE)
    recs["beg1"] = rng.integers(-2 ** 31, 2 ** 31 - 1, 2000)
    recs["end1"] = rng.integers(-2 ** 31, 2 ** 31 - 1, 2000)
    recs["len"] = rng.integers(1, 10 ** 6, 2000)
    recs["cg"] = rng.random(2000)
    # oe values at 6-decimal rounding boundaries
    recs["oe"] = np.round(rng.random(2000) * 3, 6) + 5e-7
    txt = format_islands(recs).decode()
    ref = "".join(co.format_island(r) for r in recs)
    assert txt == ref


def test_model_file_matches_restatement():
    from cpgisland_amd import HmmModel
    from cpgisland_amd.hmm import format_model
    m = HmmModel.initial()
    assert format_model(m).decode() == pr.format_model(m.to_struct())
    rng = np.random.default_rng(5)
    for scale in (1.0, 1e-4, 1e-8, 1e7, 3e-3):
        v = rng.random(104) * scale
        v[:3] = [0.0, 1e-3, 1e7]
        mm = HmmModel.from_struct(v)
        assert format_model(mm).decode() == pr.format_model(v)


@pytest.mark.parametrize("x,s", [(0.0, "0.0"), (1.0, "1.0"), (0.1, "0.1"), (1e-3, "0.001"),
                                 (1e-4, "1.0E-4"), (1e7, "1.0E7"), (1234567.0, "1234567.0"),
                                 (0.30000000000000004, "0.30000000000000004"),
                                 (2.5e-5, "2.5E-5"), (-0.5, "-0.5")])
def test_double_to_string_known_answers(x, s):
    assert pr.java_dtoa(x) == s
