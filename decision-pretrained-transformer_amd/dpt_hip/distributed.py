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


def regret_stats_allreduce(opt_local, lnr_local, n_total, group=None):
    """Suboptimality and cumulative-regret mean / SEM curves over ALL tasks of all ranks
    (evals/eval_bandit.py:169-178: diff = opt - lnr, cumsum over steps, mean and
    scipy.stats.sem with ddof=1 over tasks) from one all_reduce of per-step moments
    (4 x H fp64) instead of gathering every task's curve.  Same values as the gathered
    computation up to fp64 summation order (sum-of-squares form of the variance).
    opt_local / lnr_local: (count, H) arm-value curves of this rank's tasks."""
    diff = opt_local.to(torch.float64) - lnr_local.to(torch.float64)
    cr = torch.cumsum(diff, dim=1)
    mom = torch.stack([diff.sum(0), (diff * diff).sum(0), cr.sum(0), (cr * cr).sum(0)])
    dist.all_reduce(mom, group=group)
    n = float(n_total)

    def mean_sem(s1, s2):
        mean = s1 / n
        var = (s2 - s1 * mean) / (n - 1.0)
        return mean, torch.sqrt(torch.clamp(var, min=0.0) / n)

    sm, ss = mean_sem(mom[0], mom[1])
    rm, rsem = mean_sem(mom[2], mom[3])
    return dict(subopt_mean=sm, subopt_sem=ss, regret_mean=rm, regret_sem=rsem)
