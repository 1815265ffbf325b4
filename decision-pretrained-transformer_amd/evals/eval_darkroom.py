"""DarkRoom evaluation — drop-in for the reference evals/eval_darkroom.py.

``deploy_online_vec`` (evals/eval_darkroom.py:20-84): with the DPT controller
over this package's ``Transformer`` and a ``DarkroomEnvVec`` the whole loop is
one fused kernel launch (dpt_rollout_darkroom) when the window fits (1 + H <=
dpt_hip.darkroom_max_window(): 512 tokens) at width 32; otherwise it stays on the device step by
step (any width) — per step one window forward (gfx950 kernels) over the fixed
in-context episodes with the current state as query, device sampling, the
integer grid step kernel, and an on-device append into the episode buffers;
returns are summed on device and copied once at the end.  Other controllers
run the reference's episode loop (envs step on the device).
"""
import numpy as np
import torch

import dpt_hip
from ctrls.ctrl_darkroom import DarkroomOptPolicy, DarkroomTransformerController
from envs.darkroom_env import DarkroomEnv, DarkroomEnvPermuted, DarkroomEnvVec
from utils import convert_to_tensor

device = torch.device("cuda" if torch.cuda.is_available() else "cpu")


def _device_ok(vec_env, controller):
    """The per-step device loop: our controller, env and model.  Width 32 forwards through the packed
    device model; other widths through the generic kernels (_GenericWindow), for an inference-mode
    model (test: the last position's logits).  At every width no dropout may be in play: a
    training-mode model with dropout > 0 takes the controller's loop, whose forward applies it."""
    from models.net import Transformer
    m = controller.model
    return (isinstance(controller, DarkroomTransformerController) and isinstance(vec_env, DarkroomEnvVec)
            and isinstance(m, Transformer) and controller.batch_size == vec_env.num_envs
            and not (m.training and m.dropout > 0) and (m.n_embd == dpt_hip.E or m.test))


class _GenericWindow:
    """forward_window for a model of another width: Transformer.forward's generic kernels
    (dpt_train_forward on the forward-only workspace) over [query | context], last position."""

    def __init__(self, model):
        from dpt_hip import train as tr
        self.model = model
        self.blob = tr.pack_params(tr.param_list(model), dpt_hip.device())  # fixed for the eval

    def forward_window(self, query, cs=None, ca=None, cn=None, cr=None):
        x = {"query_states": query}
        if cs is not None:
            x.update(context_states=cs, context_actions=ca, context_next_states=cn, context_rewards=cr)
        with torch.no_grad():
            return self.model._forward_generic(x)

    def episode(self, n, ctx):
        """fwd(state, rows) -> the last-position logits of tasks ``rows`` (None: all n) with their
        current ``state`` as query: the episode's token rows (_tokens: [query | context], models/net.py
        :42-54) are packed once, and a step rewrites the query slot and gathers the rows it forwards."""
        from dpt_hip import train as tr
        m = self.model
        sd = m.state_dim
        x = {"query_states": torch.zeros((n, sd), device=dpt_hip.device())}
        if ctx:
            x.update(context_states=ctx[0], context_actions=ctx[1], context_next_states=ctx[2],
                     context_rewards=ctx[3])
        tok = m._tokens(x)
        flags = tr.FORWARD_ONLY | tr.LAST_ONLY  # _forward_generic's flags for a test-mode model without grad

        def fwd(state, rows=None):
            tok[:, 0, :sd].copy_(state)
            t = tok if rows is None else tok.index_select(0, rows)
            d = tr.desc(m.n_layer, m.n_embd, sd, m.action_dim, m.n_positions, t.shape[0], t.shape[1], flags=flags)
            return tr.forward(d, self.blob, t)[0][:, -1]
        return fwd


def _window_model(model):
    return model.device_model() if model.n_embd == dpt_hip.E else _GenericWindow(model)


def _episode_device(dm, ctrl, vec_env, ctx, horizon):
    """One DarkroomEnvVec.deploy_eval episode on device: returns (states, actions, next, rewards).

    The context is fixed for the episode, so a task's logits are a pure function of its
    query state: with dpt_hip.darkroom_memo() (default) a step forwards only the tasks
    whose current state is new in this episode and reuses the stored logits of the
    others (each task's forward is independent, so the logits are bit-identical)."""
    dev = dpt_hip.device()
    N = vec_env.num_envs
    state = torch.zeros((N, 2), dtype=torch.int32, device=dev)   # DarkroomEnv.reset -> (0, 0)
    es = torch.empty((N, horizon, 2), dtype=torch.int32, device=dev)
    ea = torch.empty((N, horizon), dtype=torch.int64, device=dev)
    er = torch.empty((N, horizon), dtype=torch.int32, device=dev)
    goals, perms, dim = vec_env.goals_device, vec_env.perms_device, vec_env.dim
    first_task = getattr(vec_env, "first_task", 0)  # draws keyed by global task id, as in rollout_fused
    memo = None
    if dpt_hip.darkroom_memo():
        memo = torch.empty((N, dim * dim, vec_env.action_dim), dtype=torch.float32, device=dev)
        seen = torch.zeros((N, dim * dim), dtype=torch.bool, device=dev)
        rows = torch.arange(N, device=dev)
    win = dm.episode(N, ctx) if hasattr(dm, "episode") else None
    for t in range(horizon):
        if memo is None:
            logits = win(state) if win else dm.forward_window(state.float(), *ctx)
        else:
            cell = state[:, 0].long() * dim + state[:, 1].long()
            need = (~seen[rows, cell]).nonzero().squeeze(1)
            if need.numel():
                cn = cell.index_select(0, need)
                if win:
                    lg = win(state, need)
                else:
                    lg = dm.forward_window(state.index_select(0, need).float(), *(c.index_select(0, need) for c in ctx))
                memo[need, cn] = lg
                seen[need, cn] = True
            logits = memo[rows, cell]
        a = ctrl.select(logits, first_task=first_task)
        es[:, t] = state
        ea[:, t] = a
        state, r = dpt_hip.darkroom_step(state, a, goals, perms, dim)
        er[:, t] = r
    ns = torch.cat([es[:, 1:], state[:, None]], dim=1)
    return es, ea, ns, er


def _fused_ok(vec_env, controller, H):
    # dpt_rollout_darkroom: 1 + H tokens per forward
    return (_device_ok(vec_env, controller) and controller.model.n_embd == dpt_hip.E
            and vec_env.state_dim == 2 and vec_env.action_dim == 5
            and 1 + H <= dpt_hip.darkroom_max_window() and vec_env.dim <= 255)


def rollout_fused(vec_env, controller, Heps, H, horizon, want_actions=False, want_logits=False,
                  want_forwards=False):
    """The whole deploy_online_vec loop as one dpt_rollout_darkroom launch.

    Selection draws are the controller's own stream: the counters this loop
    would consume step by step (one per select) are consumed here in one go,
    so the fused and per-step paths act identically on the same draws.
    """
    dm = controller.model.device_model()
    steps = Heps * horizon
    seed, ctr0 = controller._stream.next()
    controller._stream.counter = ctr0 + steps
    u = None
    if controller.sample and controller.uniforms is not None:
        u = torch.stack([torch.as_tensor(controller.uniforms(ctr0 + k), dtype=torch.float64).reshape(-1)
                         for k in range(steps)])
    return dm.rollout_darkroom(vec_env.goals_device, Heps, horizon, H // horizon, dim=vec_env.dim,
                               perms=vec_env.perms_device, sample=controller.sample, temp=controller.temp,
                               seed=seed, counter=ctr0, first_task=getattr(vec_env, "first_task", 0), uniforms=u,
                               want_actions=want_actions, want_logits=want_logits, want_forwards=want_forwards)


def deploy_online_vec(vec_env, controller, Heps, H, horizon, fused=True):
    assert H % horizon == 0
    if fused and _fused_ok(vec_env, controller, H):
        # the fused kernel holds the model's parameter block in LDS next to the window's K/V; a
        # deep model whose block does not fit beside a long window is refused (DPT_EUNSUPPORTED ->
        # NotImplementedError) before anything ran or any draw was consumed: take the per-step loop
        ctr = controller._stream.counter
        try:
            return rollout_fused(vec_env, controller, Heps, H, horizon)["returns"].to(torch.int64).cpu().numpy()
        except NotImplementedError:
            controller._stream.counter = ctr
    ctx_rollouts = H // horizon
    num_envs = vec_env.num_envs
    dev = dpt_hip.device()
    sd, ad = vec_env.state_dim, vec_env.action_dim
    cs = torch.zeros((num_envs, ctx_rollouts, horizon, sd), device=dev)
    ca = torch.zeros((num_envs, ctx_rollouts, horizon, ad), device=dev)
    cn = torch.zeros((num_envs, ctx_rollouts, horizon, sd), device=dev)
    cr = torch.zeros((num_envs, ctx_rollouts, horizon, 1), device=dev)
    fast = _device_ok(vec_env, controller)
    dm = _window_model(controller.model) if fast else None
    cum_means = []
    for ep in range(Heps):
        if ep < ctx_rollouts:
            ctx = [x[:, :ep].reshape(num_envs, -1, x.shape[-1]) for x in (cs, ca, cn, cr)]
        else:  # the last ctx_rollouts episodes (shift-append, eval_darkroom.py:75-82)
            ctx = [x.reshape(num_envs, -1, x.shape[-1]) for x in (cs, ca, cn, cr)]
        if fast:
            c = () if ctx[0].shape[1] == 0 else (ctx[0], ctx[1], ctx[2], ctx[3][..., 0])
            es, ea, ens, er = _episode_device(dm, controller, vec_env, c, horizon)
            new = (es.float(), torch.nn.functional.one_hot(ea, ad).float(), ens.float(), er.float()[..., None])
            cum_means.append(er.sum(-1))
        else:
            batch = {"context_states": ctx[0], "context_actions": ctx[1], "context_next_states": ctx[2],
                     "context_rewards": ctx[3]}
            controller.set_batch(batch)
            s, a, n, r = vec_env.deploy_eval(controller)
            cum_means.append(torch.as_tensor(np.sum(r, axis=-1), device=dev))
            new = (convert_to_tensor(s), convert_to_tensor(a), convert_to_tensor(n), convert_to_tensor(r[:, :, None]))
        if ep < ctx_rollouts:
            for buf, v in zip((cs, ca, cn, cr), new):
                buf[:, ep] = v
        else:
            cs, ca, cn, cr = (torch.cat((buf[:, 1:], v[:, None]), dim=1) for buf, v in zip((cs, ca, cn, cr), new))
    return torch.stack(cum_means, dim=1).cpu().numpy()


def online(eval_trajs, model, Heps, H, n_eval, dim, horizon, permuted=False):
    """evals/eval_darkroom.py:87-121."""
    import matplotlib.pyplot as plt
    import scipy.stats
    assert H % horizon == 0
    envs = []
    for i in range(n_eval):
        traj = eval_trajs[i]
        envs.append(DarkroomEnvPermuted(dim, traj["perm_index"], horizon) if permuted
                    else DarkroomEnv(dim, traj["goal"], horizon))
    lnr = DarkroomTransformerController(model, batch_size=n_eval, sample=True)
    vec_env = DarkroomEnvVec(envs)
    all_means_lnr = np.array(deploy_online_vec(vec_env, lnr, Heps, H, horizon))
    means_lnr = np.mean(all_means_lnr, axis=0)
    sems_lnr = scipy.stats.sem(all_means_lnr, axis=0)
    for i in range(n_eval):
        plt.plot(all_means_lnr[i], color="blue", alpha=0.2)
    plt.plot(means_lnr, label="Learner")
    plt.fill_between(np.arange(Heps), means_lnr - sems_lnr, means_lnr + sems_lnr, alpha=0.2)
    plt.legend()
    plt.xlabel("Episodes")
    plt.ylabel("Average Return")
    plt.title(f"Online Evaluation on {n_eval} Envs")
    return all_means_lnr


def offline(eval_trajs, model, n_eval, H, dim, permuted=False, uniforms=None):
    """evals/eval_darkroom.py:124-189: expert vs DPT (sampled and greedy) on fixed contexts.
    ``uniforms`` (H, n_eval), optional: the sampled leg's selection draws (one row per step), as
    the reference's np.random.choice consumes them; returns the three per-task return arrays."""
    import matplotlib.pyplot as plt
    envs = []
    for i in range(n_eval):
        traj = eval_trajs[i]
        envs.append(DarkroomEnvPermuted(dim, traj["perm_index"], H) if permuted else DarkroomEnv(dim, traj["goal"], H))
    trajs = eval_trajs[:n_eval]
    vec_env = DarkroomEnvVec(envs)
    opt = _OptVec(envs)
    _, _, _, rs_opt = vec_env.deploy_eval(opt)
    batch = {"context_states": convert_to_tensor([t["context_states"] for t in trajs]),
             "context_actions": convert_to_tensor([t["context_actions"] for t in trajs]),
             "context_next_states": convert_to_tensor([t["context_next_states"] for t in trajs]),
             "context_rewards": convert_to_tensor([t["context_rewards"][:, None] for t in trajs])}
    res = {"Opt": np.sum(rs_opt, axis=-1)}
    for name, sample in (("Learner", True), ("Learner (greedy)", False)):
        ctrl = DarkroomTransformerController(model, batch_size=n_eval, sample=sample)
        if sample and uniforms is not None:
            ctrl.uniforms = lambda k: uniforms[k]
        ctrl.set_batch(dict(batch))
        if _device_ok(vec_env, ctrl):
            c = (batch["context_states"], batch["context_actions"], batch["context_next_states"],
                 batch["context_rewards"][..., 0])
            _, _, _, er = _episode_device(_window_model(model), ctrl, vec_env, c, H)
            res[name] = er.sum(-1).cpu().numpy()
        else:  # other widths / model classes: the controller's own per-step forward
            _, _, _, rs = vec_env.deploy_eval(ctrl)
            res[name] = np.sum(rs, axis=-1)
    means = {k: np.mean(v) for k, v in res.items()}
    colors = plt.cm.viridis(np.linspace(0, 1, len(means)))
    plt.bar(means.keys(), means.values(), color=colors)
    plt.ylabel("Average Return")
    plt.title(f"Average Return on {n_eval} Trajectories")
    return res


class _OptVec:
    """Vectorised DarkroomOptPolicy over a DarkroomEnvVec (one device kernel per step)."""

    def __init__(self, envs):
        self.envs = envs
        self.vec = DarkroomEnvVec(envs)

    def act(self, states):
        st = np.stack([np.asarray(s, np.int32) for s in states])
        a = dpt_hip.darkroom_opt_action(st, self.vec.goals_device, self.vec.perms_device).cpu().numpy()
        return np.eye(5)[a]


__all__ = ["deploy_online_vec", "online", "offline", "DarkroomOptPolicy"]
