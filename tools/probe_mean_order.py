"""Which summation order / projection torch's .mean(-1) over a contiguous [B, n] fp32 tensor uses
on this device (diagnostic for the fused kernels' ordered_sum, simulator/_fused.py)."""
import torch


def strided(v, s):
    acc = []
    for i in range(min(s, len(v))):
        a = v[i]
        for j in range(i + s, len(v), s):
            a = a + v[j]
        acc.append(a)
    return acc


def seq(v):
    s = v[0]
    for t in v[1:]:
        s = s + t
    return s


def tree(v):
    v = list(v)
    w = 1
    while w < len(v):
        for i in range(0, len(v) - w, 2 * w):
            v[i] = v[i] + v[i + w]
        w *= 2
    return v[0]


dev = torch.device("cuda")
for n in range(2, 17):
    g = torch.Generator(device="cpu").manual_seed(1234 + n)
    x = (torch.rand(4096, n, generator=g) * torch.exp2(torch.randint(-12, 12, (4096, n), generator=g).float())).to(dev)
    ref = x.mean(-1)
    refsum = x.sum(-1)
    cols = [x[:, i] for i in range(n)]
    cands = {"seq": seq(cols), "rev": seq(cols[::-1]), "tree": tree(cols)}
    for s in (2, 4, 8):
        a = strided(cols, s)
        cands[f"str{s}_seq"] = seq(a)
        cands[f"str{s}_tree"] = tree(a)
    hits = []
    for k, v in cands.items():
        if torch.equal(v * (1.0 / n), ref):
            hits.append(k + "*inv")
        if torch.equal(v / n, ref):
            hits.append(k + "/n")
        if torch.equal(v, refsum):
            hits.append(k + "=sum")
    print(n, hits, flush=True)
