"""Task sharding over GPUs.

Tasks never interact, so the rollout itself has no collective: each rank runs
its contiguous block of tasks (Philox keyed by the GLOBAL task id, so results
do not depend on the number of ranks) and the per-task curves are gathered
once with ``all_gather_into_tensor`` (RCCL over xGMI with the ``nccl``
backend; ``gloo`` in CPU tests).  Uneven blocks are padded to the largest.
"""
import torch
import torch.distributed as dist


def shard(n_total, world, rank):
    """Contiguous block of tasks for ``rank``: (first_task, count)."""
    base, rem = divmod(n_total, world)
    first = rank * base + min(rank, rem)
    return first, base + (1 if rank < rem else 0)


def gather_rows(local, n_total, group=None):
    """All-gather per-task rows (count, ...) from every rank into (n_total, ...) on every rank."""
    world = dist.get_world_size(group)
    counts = [shard(n_total, world, r)[1] for r in range(world)]
    width = max(counts)
    pad = torch.zeros((width,) + tuple(local.shape[1:]), dtype=local.dtype, device=local.device)
    pad[: local.shape[0]] = local
    out = torch.empty((world * width,) + tuple(local.shape[1:]), dtype=local.dtype, device=local.device)
    if dist.get_backend(group) == "gloo":  # CPU tests / one-GPU rehearsal: gather on the host
        host = pad.cpu()
        parts = [torch.empty_like(host) for _ in range(world)]
        dist.all_gather(parts, host, group=group)
        out = torch.cat(parts).to(local.device)
    else:
        dist.all_gather_into_tensor(out, pad, group=group)
    return torch.cat([out[r * width: r * width + counts[r]] for r in range(world)])


def sharded_online(rollout_fn, means_all, group=None):
    """Run ``rollout_fn(means_local, first_task) -> dict with 'arm_value' (count, H)`` on this
    rank's block and gather the (N_total, H) arm-value curves (the regret inputs) everywhere."""
    world, rank = dist.get_world_size(group), dist.get_rank(group)
    n_total = means_all.shape[0]
    first, count = shard(n_total, world, rank)
    out = rollout_fn(means_all[first:first + count], first)
    return gather_rows(out["arm_value"], n_total, group), out


def _all_reduce(t, group=None):
    """Sum ``t`` over ranks in place (RCCL for device tensors under ``nccl``; under ``gloo``, the
    CPU tests' and the one-GPU rehearsal's backend, a device tensor goes through the host)."""
    if t.is_cuda and dist.get_backend(group) == "gloo":
        host = t.cpu()
        dist.all_reduce(host, group=group)
        t.copy_(host)
    else:
        dist.all_reduce(t, group=group)


def _regret_max_steps():
    import dpt_hip
    return dpt_hip.regret_max_steps()


def regret_stats_allreduce(opt_local, lnr_local, n_total, group=None):
    """Suboptimality and cumulative-regret mean / SEM curves over ALL tasks of all ranks
    (evals/eval_bandit.py:169-178: diff = opt - lnr, cumsum over steps, mean and
    scipy.stats.sem with ddof=1 over tasks) without gathering every task's curve.

    Two all_reduces of 2 x H fp64: the per-step sums give the global means, then each
    rank sums its squared deviations from those means (the centred two-pass form
    scipy uses, so a large mean relative to the spread loses nothing to cancellation,
    as the sum-of-squares form would).  Equal to scipy.stats.sem over the gathered
    curves up to fp64 summation order.
    opt_local / lnr_local: (count, H) (or broadcastable (count, 1)) arm-value curves of this
    rank's tasks.  Without an initialised process group it is the single-process statistic.
    fp64 curves on the GPU take the device passes (dpt_regret_moments); others the torch ops."""
    distributed = dist.is_available() and dist.is_initialized()  # else: one process holds every task
    n = float(n_total)
    count, H = lnr_local.shape[0], lnr_local.shape[1]
    if count == 0:
        # a rank with no tasks (shard() gives n_total < world ranks one task each): it adds
        # zero moments but still joins both all_reduces, so the other ranks never block
        s1 = torch.zeros((2, H), dtype=torch.float64, device=lnr_local.device)
        if distributed:
            _all_reduce(s1, group)
        mean = s1 / n
        m2 = torch.zeros_like(s1)
    elif lnr_local.is_cuda and lnr_local.dtype == torch.float64 and H <= _regret_max_steps():
        # device passes (dpt_regret_moments, HIP): one read of the curves each
        import dpt_hip
        opt = opt_local.reshape(count, -1)[:, 0].contiguous()
        s1 = dpt_hip.regret_moments(lnr_local, opt)
        if distributed:
            _all_reduce(s1, group)
        mean = s1 / n
        m2 = dpt_hip.regret_moments(lnr_local, opt, dpt_hip._lib.REGRET_CENTRED, mean)
    else:
        diff = opt_local.to(torch.float64) - lnr_local.to(torch.float64)
        cr = torch.cumsum(diff, dim=1)
        s1 = torch.stack([diff.sum(0), cr.sum(0)])
        if distributed:
            _all_reduce(s1, group)
        mean = s1 / n
        m2 = torch.stack([((diff - mean[0]) ** 2).sum(0), ((cr - mean[1]) ** 2).sum(0)])
    if distributed:
        _all_reduce(m2, group)
    sem = torch.sqrt(m2 / (n - 1.0) / n)
    return dict(subopt_mean=mean[0], subopt_sem=sem[0], regret_mean=mean[1], regret_sem=sem[1])
