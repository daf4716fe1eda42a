"""The choice rule of nxec_batch_layout_tuned (nxec_layout_choose, include/
nxec.h §3): the table's layout is the incumbent and stays
unless a challenger beats it in every interleaved round by more than the
spread between those rounds -- box-to-box and call-to-call drift of 2-3 %
(profiles/r05_configs_box_{a,b}.jsonl) must not replace a good static
layout with a worse measured one.  Pure host logic: no device."""
import ctypes as C

from nexoedge_amd import _lib

L = _lib.lib


def choose(rounds, margin=0.005):
    """rounds: [[score of candidate c in round r]]"""
    nc, nr = len(rounds[0]), len(rounds)
    flat = (C.c_double * (nc * nr))(*[v for r in rounds for v in r])
    return L.nxec_layout_choose(nc, nr, flat, C.c_double(margin))


def test_tie_keeps_the_incumbent():
    assert choose([[100.0, 100.0], [100.0, 100.0], [100.0, 100.0]]) == 0
    assert choose([[100.0]]) == 0  # the incumbent is always a candidate


def test_challenger_must_win_every_round():
    # +3 % in two rounds, -1 % in the third: not a consistent win
    assert choose([[100, 103], [100, 103], [100, 99]]) == 0
    # +3 % in every round, rounds agree: replaced
    assert choose([[100, 103], [100, 103.2], [100, 102.9]]) == 1


def test_margin_is_the_measured_spread():
    # the incumbent's rounds spread 4 %: a steady +3 % challenger is noise
    assert choose([[98, 101], [102, 105], [100, 103]]) == 0
    # the same challenger beats a steady incumbent
    assert choose([[100, 103], [100, 103.1], [100, 103.05]]) == 1
    # below the 0.5 % floor even with no spread
    assert choose([[100, 100.4], [100, 100.4], [100, 100.4]]) == 0


def test_best_of_the_winners_not_the_first():
    # table 100, A +0.6 %, B +1 % -- B (argmax), not A
    assert choose([[100, 100.6, 101.0]] * 3, margin=0.005) == 2
    # a challenger with the highest mean but one losing round is skipped
    assert choose([[100, 102, 110], [100, 102, 99], [100, 102, 110]]) == 1


def test_unmeasured_candidates_are_skipped():
    assert choose([[100, 0, 103], [100, 0, 103], [100, 0, 103]]) == 2
    assert choose([[0, 150], [100, 150], [100, 150]]) == 0  # incumbent unmeasured in a round: keep it


def test_bad_arguments():
    assert L.nxec_layout_choose(0, 3, None, C.c_double(0.0)) == _lib.NXEC_ERR_INVALID
    one = (C.c_double * 1)(1.0)
    assert L.nxec_layout_choose(1, 1, one, C.c_double(-1.0)) == _lib.NXEC_ERR_INVALID
