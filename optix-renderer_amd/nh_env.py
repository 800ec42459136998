"""Process environment the HIP runtime reads once, at its initialisation (no library is loaded here).

The wavefront pipeline drives up to three path pools on their own streams; each needs its own hardware queue, or
one pool's long tail kernel blocks another's bounces (HIP's default is 4 queues per process, one of which the
context's own stream takes; the MI355X boxes export that 4 explicitly: C1 -15 %, profiles/round4_session3_ab.txt).
Shared by the binding (`nori_hip`, at import) and `bench.py` (before torch may initialise HIP).
"""
import os

HW_QUEUES_MIN = 8


def parse_hw_queues(value):
    """GPU_MAX_HW_QUEUES as an int; unset, empty or non-numeric values read as 0 (HIP's own default applies)."""
    try:
        return int(value or 0)
    except (TypeError, ValueError):
        return 0


def raise_hw_queues(minimum=HW_QUEUES_MIN):
    """Raise GPU_MAX_HW_QUEUES to `minimum` unless a larger value is set or NH_KEEP_HW_QUEUES asks to keep it.

    Has an effect only before the process's first HIP call. Returns the value the runtime will see."""
    cur = parse_hw_queues(os.environ.get("GPU_MAX_HW_QUEUES"))
    if cur < minimum and not os.environ.get("NH_KEEP_HW_QUEUES"):
        os.environ["GPU_MAX_HW_QUEUES"] = str(minimum)
        return minimum
    return cur
