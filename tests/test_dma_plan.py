"""CPU check of the conv kernels' LDS-DMA piece plans and tap addressing
(tools/check/dma_plan.py): every piece issued once, every source and LDS
destination in bounds, every tap read seeing the reference im2col's input byte
(RK/kernels/im2col.cu:37-54) or a zero, for ragged and full batches."""
import os
import re
import sys

import pytest

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "tools", "check"))
import dma_plan  # noqa: E402

ROOT = os.path.join(os.path.dirname(__file__), "..")


@pytest.mark.parametrize("N", [1, 2, 3, 5, 17, 256])
def test_dma_plans(N):
    dma_plan.run([N])


def test_checker_catches_a_wrong_tap():
    """The checker is not vacuous: shifting the stride-2 patch rows by one
    input row makes it fail."""
    orig = dma_plan.check_s2i
    src = open(dma_plan.__file__).read()
    bad = src.replace('ih = 2 * (gr - n * g["OH"]) - 1 + r', 'ih = 2 * (gr - n * g["OH"]) + r')
    assert bad != src
    ns = {}
    exec(compile(bad, "dma_plan_mutant", "exec"), ns)
    with pytest.raises(ns["Fail"]):
        ns["check_s2i"](14, 2)
    assert dma_plan.check_s2i is orig


def test_engine_batch_limit_keeps_int32_offsets():
    """The engine refuses batches past the int32 offset bound the plans rely on."""
    src = open(os.path.join(ROOT, "dlq_amd", "csrc", "dlq_internal.h")).read()
    m = re.search(r"constexpr int kMaxBatch = (\d+);", src)
    assert m, "kMaxBatch not declared"
    assert int(m.group(1)) <= dma_plan.max_batch_int32()
