import cProfile, pstats, io, os, sys, numpy as np, torch
ROOT = os.environ.get("GRAFT_REPO_ROOT", "/root/repo")
sys.path[:0] = [os.path.join(ROOT, "decision-pretrained-transformer_amd"), ROOT, os.path.join(ROOT, "scripts")]
from models.net import Transformer
from train_timing import batch
dev = torch.device("cuda")
sd, A, H = 2, 5, 100
m = Transformer(dict(horizon=H, state_dim=sd, action_dim=A, n_layer=4, n_embd=32, n_head=1, dropout=0.0, test=False)).to(dev).train()
b = batch(64, H, sd, A, dev, np.random.RandomState(0))
ce = torch.nn.CrossEntropyLoss(reduction="sum")
opt = torch.optim.AdamW(m.parameters(), lr=1e-4, weight_decay=1e-4)
true = b["optimal_actions"][:, None, :].expand(64, H, A).reshape(-1, A)
def step():
    pred = m(b); loss = ce(pred.reshape(-1, A), true); opt.zero_grad(); loss.backward(); opt.step()
for _ in range(5): step()
torch.cuda.synchronize()
pr = cProfile.Profile(); pr.enable()
for _ in range(50): step()
pr.disable(); torch.cuda.synchronize()
s = io.StringIO(); pstats.Stats(pr, stream=s).sort_stats("tottime").print_stats(30); print(s.getvalue())
s = io.StringIO(); pstats.Stats(pr, stream=s).sort_stats("cumtime").print_stats(30); print(s.getvalue())
