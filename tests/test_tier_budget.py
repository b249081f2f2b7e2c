"""The multigpu tier's wall bound (tests/_mp.py TierBudget): however many
launches the tier has and however each ends, the launches' bounds sum to at
most the tier budget, so single-GPU tests (<= 300 s) + the tier stay inside
the driver's 900 s `pytest -m gpu` step cap."""
from tests._mp import MAX_TIMEOUT, TierBudget


class _Clock:
    def __init__(self):
        self.t = 1000.0

    def __call__(self):
        return self.t


def _worst_case(budget, launches, min_launch=30.0):
    clk = _Clock()
    tb = TierBudget(budget, min_launch=min_launch, clock=clk)
    used, ran, skipped = 0.0, 0, 0
    for _ in range(launches):
        t = tb.next_timeout()
        if t is None:
            skipped += 1
            clk.t += 0.5  # a skip costs nothing but the test's own overhead
            continue
        assert 0 < t <= MAX_TIMEOUT
        clk.t += t  # every launch runs into its bound
        used += t
        ran += 1
    return used, ran, skipped


def test_tier_worst_case_is_the_budget():
    for budget in (60.0, 300.0, 480.0, 550.0):
        for launches in (1, 3, 10, 40):
            used, ran, skipped = _worst_case(budget, launches)
            assert used <= budget + 1e-9, (budget, launches, used)
            assert ran + skipped == launches


def test_default_tier_fits_the_driver_cap():
    """10 launches of the default tier, each hitting its bound, after 300 s of
    single-GPU tests: inside 850 s (the 900 s cap minus teardown slack)."""
    import os

    budget = float(os.environ.get("IGG_MGPU_TIER_BUDGET", "480"))
    used, ran, skipped = _worst_case(budget, 10)
    assert 300.0 + used <= 850.0, used
    assert ran >= 2  # the first, most valuable launches always get their full bound


def test_first_launch_starts_the_clock():
    clk = _Clock()
    tb = TierBudget(100.0, clock=clk)
    clk.t += 5000.0  # collection and the single-GPU tests before the tier
    assert tb.next_timeout() == min(MAX_TIMEOUT, 100.0)
