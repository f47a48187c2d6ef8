"""Bounded Adam grid of ranks sharing one GPU (fedmi.parallel.peer.shared_adam_grid): sized from
the device's resident-workgroup slots, not a hard-coded MI355X CU count."""
from fedmi.parallel.peer import SHARED_GPU_ADAM_SLOTS, adam_slots, shared_adam_grid


def test_full_grid_when_every_rank_fits():
    assert shared_adam_grid(1, 179) == 0                 # one rank per GPU: always the full grid
    assert shared_adam_grid(2, 100, slots=256) == 0      # 200 <= 256 resident workgroups
    assert shared_adam_grid(8, 179, slots=256) == 16     # the world-8 shared-GPU test's grid


def test_small_device_bounds_the_grid():
    # e.g. a CPX partition (32 CUs): 2 x 20 blocks no longer fit, each rank gets 16 / 2 = 8
    assert shared_adam_grid(2, 20, slots=32) == 8
    assert shared_adam_grid(8, 179, slots=32) == 2
    assert shared_adam_grid(8, 179, slots=8) == 1        # never 0 workgroups
    # every rank's bounded grid fits on the device at once
    for slots in (8, 32, 80, 256):
        for n in range(2, 9):
            g = shared_adam_grid(n, 179, slots=slots)
            assert g >= 1 and (n * g <= slots or g == 1)


def test_slots_without_a_device():
    assert adam_slots(None) == SHARED_GPU_ADAM_SLOTS
