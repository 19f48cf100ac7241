"""Host-side scratch-buffer plumbing of the rasterizer (CPU only, no library call)."""
import gc
import weakref

import pytest
import torch

from gaussian_splatting_lightning_amd.rasterizer import _Buffers


def test_buffers_are_freed_without_the_cyclic_collector():
    """The allocation callback must not tie the buffer holder into a reference cycle: with the cyclic
    collector disabled (bench.py's timed region) every call's buffers would otherwise stay alive, and at
    5M Gaussians / 4K the device ran out of memory after a few dozen steps."""
    was = gc.isenabled()
    gc.disable()
    try:
        b = _Buffers(torch.device("cpu"))
        ptr = b.callback(None, 1, 4096)
        assert ptr and b.get(1).numel() == 4096
        ref_holder, ref_buf = weakref.ref(b), weakref.ref(b.get(1))
        del b
        assert ref_holder() is None
        assert ref_buf() is None
    finally:
        if was:
            gc.enable()


def test_failed_allocation_returns_null_and_reraises():
    """An exception inside the callback (out of memory) becomes a NULL return -- which the library reports as
    GSR_ERR_ALLOC -- and is re-raised by the caller after the call."""
    b = _Buffers(torch.device("cpu"))
    assert not b.callback(None, 2, 1 << 62)
    assert b.get(2).numel() == 0
    with pytest.raises(RuntimeError):
        b.raise_pending()
