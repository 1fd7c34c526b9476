"""GPU: orpcd_gicp_batch_window -- a GICP batch run over a window of passes,
its running starts resumed later from their state (the multi-GPU re-deal of
running starts).  Resuming a start -- in a batch of another
size and order, on another context, against a multi-target set -- continues
it bit for bit: T, rmse, fitness, iterations and correspondences equal the
uninterrupted batch's."""
import numpy as np
import pytest

from workloads import rot_xyz, small_pair

pytestmark = pytest.mark.gpu

KEYS = ("T", "rmse", "fitness", "iters", "ncorr")


def _starts(B, seed):
    rng = np.random.default_rng(seed)
    return np.array([rot_xyz(*rng.uniform(-60, 60, 3)) for _ in range(B)]), rng.normal(size=(B, 3)) * 0.05


@pytest.mark.parametrize("B,P", [(20, 6), (20, 1), (8, 3)])
def test_window_then_resume_is_the_uninterrupted_batch(B, P):
    from orpcd_amd import _native
    src, tgt = small_pair(6007, 5003, seed=11)
    R0, t0 = _starts(B, B + P)
    a, b = _native.Context(0), _native.Context(0)
    for c in (a, b):
        c.set_target(tgt, 1e-3)
        c.set_source(src)
    full = a.gicp_batch(R0, t0, max_correspondence_distance=0.3)
    w = a.gicp_batch_window(R0, t0, pass_end=P, max_correspondence_distance=0.3)
    done = w["done"]
    for k in KEYS:
        assert np.array_equal(w[k][done], full[k][done]), k
    run = np.nonzero(~done)[0]
    assert len(run) > 2, "the window should leave starts running"
    # the running starts, reversed and split over two batches on the other context
    halves = [run[::-1][: len(run) // 2], run[::-1][len(run) // 2:]]
    for h in halves:
        r = b.gicp_batch_window(R0[h], t0[h], pass_begin=P, state=w["state"][h], max_correspondence_distance=0.3)
        assert r["done"].all()
        for k in KEYS:
            assert np.array_equal(r[k], full[k][h]), k
    for c in (a, b):
        c.close()


def test_window_multi_target_resume():
    from orpcd_amd import _native
    src, tgt = small_pair(6007, 5003, seed=12)
    tgts = [tgt, tgt * np.array([1.05, 1.0, 0.95])]
    R0, t0 = _starts(18, 3)
    tos = np.array([k % 2 for k in range(18)], np.int32)
    c = _native.Context(0)
    c.set_targets(tgts, 1e-3)
    c.set_source(src)
    full = c.gicp_batch_targets(R0, t0, tos, max_correspondence_distance=0.3)
    w = c.gicp_batch_window(R0, t0, tos, pass_end=5, max_correspondence_distance=0.3)
    run = np.nonzero(~w["done"])[0]
    r = c.gicp_batch_window(R0[run], t0[run], tos[run], pass_begin=5, state=w["state"][run],
                            max_correspondence_distance=0.3)
    for k in KEYS:
        assert np.array_equal(r[k], full[k][run]), k
        assert np.array_equal(w[k][w["done"]], full[k][w["done"]]), k
    with pytest.raises(ValueError, match="pass window"):
        c.gicp_batch_window(R0, t0, tos, pass_begin=5)      # no state
    c.close()


def test_target_layouts_moved_between_contexts_bit_identical():
    """orpcd_get_target_layout / orpcd_set_target_layouts: targets built by one
    context (orpcd_set_targets) and adopted by another from device buffers give
    the same batch results bit for bit (the re-deal moves layouts between
    ranks instead of building them again); a foreign buffer is refused;
    another epsilon rebuilds the covariances from the adopted layout."""
    from orpcd_amd import _native
    src, tgt = small_pair(6007, 5003, seed=11)
    targets = [tgt, tgt * np.array([1.1, 1.0, 0.9]), tgt * np.array([0.95, 1.05, 1.0])]
    a, b = _native.Context(0), _native.Context(0)
    a.set_targets(targets, 1e-3, cache=False)
    bufs = []
    for k in range(len(targets)):
        n = a.target_layout_bytes(k)
        ptr = a.device_alloc(n)
        a.get_target_layout(k, ptr, n)
        bufs.append((n, ptr))
    with pytest.raises(ValueError):                   # smaller than the layout
        a.get_target_layout(0, bufs[0][1], bufs[0][0] - 1)
    b.set_target_layouts([p for _, p in bufs[::-1]])  # another order: targets 2, 1, 0
    R0, t0 = _starts(12, 5)
    tos = (np.arange(12) % 3).astype(np.int32)
    for c in (a, b):
        c.set_source(src, cache=False)
    prm = dict(max_correspondence_distance=0.3)
    ra = a.gicp_batch_window(R0, t0, tos, **prm)
    rb = b.gicp_batch_window(R0, t0, (2 - tos).astype(np.int32), **prm)
    for k in KEYS:
        assert np.array_equal(ra[k], rb[k]), k
    with pytest.raises(ValueError):                   # not a layout: a layout's point section
        b.set_target_layouts([bufs[0][1] + 256 * ((bufs[0][0] // 2) // 256)])
    b.set_target_layouts([p for _, p in bufs])
    prm = dict(max_correspondence_distance=0.3, epsilon=1e-2)  # covariances for another epsilon
    ra = a.gicp_batch_window(R0, t0, tos, **prm)
    rb = b.gicp_batch_window(R0, t0, tos, **prm)
    for k in KEYS:
        assert np.array_equal(ra[k], rb[k]), k
    for _, p in bufs:
        a.device_free(p)
    a.close()
    b.close()
