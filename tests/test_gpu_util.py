"""swarm_tensor_list_copy (include/swarmtrain.h): word-exact multi-tensor copy, skipped
by a device flag — the OC2 update's KL rollback (learned_option_critic_trainer.py)."""

import ctypes as C

import pytest
import torch

pytestmark = pytest.mark.gpu


def test_tensor_list_copy_exact_and_flag(gpu_device):
    from SwarmACB_isaac import _native

    lib = _native.load()
    g = torch.Generator(device=gpu_device).manual_seed(3)
    sizes = [1, 7, 256, 1000, 70_000, 3]
    src = [torch.randn(n, device=gpu_device, generator=g) for n in sizes]
    src[0].fill_(-0.0)                                   # signed zero and NaN move as words
    src[1][2] = float("nan")
    dst = [torch.zeros_like(t) for t in src]
    i64 = dict(dtype=torch.int64, device=gpu_device)
    dp = torch.tensor([t.data_ptr() for t in dst], **i64)
    sp = torch.tensor([t.data_ptr() for t in src], **i64)
    words = torch.tensor(sizes, **i64)
    flag = torch.ones((), dtype=torch.uint8, device=gpu_device)
    st = C.c_void_p(torch.cuda.current_stream(gpu_device).cuda_stream)
    p = lambda t: C.c_void_p(t.data_ptr())   # noqa: E731
    assert lib.swarm_tensor_list_copy(len(sizes), p(dp), p(sp), p(words), max(sizes), p(flag), st) == 0
    torch.cuda.synchronize(gpu_device)
    assert all(bool((d == 0).all()) for d in dst)        # flag set: nothing copied
    flag.zero_()
    assert lib.swarm_tensor_list_copy(len(sizes), p(dp), p(sp), p(words), max(sizes), p(flag), st) == 0
    torch.cuda.synchronize(gpu_device)
    for d, s in zip(dst, src):
        assert torch.equal(d.view(torch.int32), s.view(torch.int32))
