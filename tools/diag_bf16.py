import sys, torch
sys.path[:0] = ['tests', 'tests/golden']
from fixture_io import Fixture
fx = Fixture('tests/golden/fedadam_mixed_rounds.npz')
cur = fx.weights("r0/cur")["bf"]; avg = fx.weights("r1/avg")["bf"]; exp = fx.weights("r1/cur")["bf"]
b1, b2, eta, tau = 0.9, 0.99, 1e-2, 1e-3
def seq(avg, cur):
    out = {}
    d = avg - cur; out["d"] = d
    m = b1 * torch.zeros_like(d) + (1 - b1) * d; out["m"] = m
    d2 = d**2; out["d2"] = d2
    v = b2 * torch.zeros_like(d) + (1 - b2) * d2; out["v"] = v
    sq = torch.sqrt(v); out["sqrt"] = sq
    den = sq + tau; out["den"] = den
    num = eta * m; out["num"] = num
    q = num / den; out["q"] = q
    out["cur"] = cur + q
    return out
c = seq(avg, cur); g = seq(avg.cuda(), cur.cuda())
for k in c:
    diff = (c[k].float() != g[k].cpu().float())
    print(k, int(diff.sum()), c[k][diff][:4].tolist(), g[k].cpu()[diff][:4].tolist())
print("ref vs cpu", int((c["cur"] != exp).sum()), "ref vs gpu", int((g["cur"].cpu() != exp).sum()))
