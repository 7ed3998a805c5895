#!/usr/bin/env python3
"""Which rounding does torch's device Adam use?  Runs the foreach ops
torch.optim.Adam issues (_foreach_lerp_, _foreach_mul_, _foreach_addcmul_,
_foreach_sqrt, _foreach_div_, _foreach_add_, _foreach_addcdiv_) on random
f32 data on the GPU and reports, per op, the fraction of elements equal to
each candidate formula evaluated on the host (separate roundings vs one fma,
emulated in f64 then rounded).  Informs csrc/train.hip's adam_kernel."""
import json

import numpy as np
import torch


def f32(x):
    return np.asarray(x, dtype=np.float32)


def fma(a, b, c):
    return f32(np.float64(a) * np.float64(b) + np.float64(c))


def frac(a, b):
    return float(np.mean(f32(a) == f32(b)))


def main():
    n = 1 << 20
    g = torch.Generator().manual_seed(0)
    m = torch.randn(n, generator=g) * 0.3
    gr = torch.randn(n, generator=g) * 0.3
    v = torch.rand(n, generator=g) * 0.1
    p = torch.randn(n, generator=g)
    res = {}
    w = f32(1 - 0.9)
    # lerp
    d = [m.cuda()]
    torch._foreach_lerp_(d, [gr.cuda()], 1 - 0.9)
    out = d[0].cpu().numpy()
    M, G = m.numpy(), gr.numpy()
    res["lerp"] = {"sep": frac(out, f32(M + f32(w * f32(G - M)))), "fma": frac(out, fma(w, f32(G - M), M))}
    # mul + addcmul
    b2, c2 = f32(0.999), f32(1 - 0.999)
    d = [v.cuda()]
    torch._foreach_mul_(d, 0.999)
    vm = d[0].cpu().numpy()
    res["mul"] = {"sep": frac(vm, f32(v.numpy() * b2))}
    torch._foreach_addcmul_(d, [gr.cuda()], [gr.cuda()], 1 - 0.999)
    out = d[0].cpu().numpy()
    gg = f32(G * G)
    res["addcmul"] = {"sep_s(gg)": frac(out, f32(vm + f32(c2 * gg))), "fma_s(gg)": frac(out, fma(c2, gg, vm)),
                      "sep_(sg)g": frac(out, f32(vm + f32(f32(c2 * G) * G))),
                      "fma_(sg)g": frac(out, fma(f32(c2 * G), G, vm))}
    # sqrt / div / add
    V = vm
    s = torch._foreach_sqrt([torch.from_numpy(V).cuda()])
    sq = s[0].cpu().numpy()
    res["sqrt"] = {"sep": frac(sq, f32(np.sqrt(np.float64(V))))}
    bc = f32(np.sqrt(1 - 0.999 ** 3))
    torch._foreach_div_(s, [float(np.sqrt(1 - 0.999 ** 3))])
    dv = s[0].cpu().numpy()
    res["div"] = {"sep": frac(dv, f32(sq / bc)), "mul_recip": frac(dv, f32(sq * f32(1 / bc)))}
    torch._foreach_add_(s, 1e-15)
    den = s[0].cpu().numpy()
    res["add_eps"] = {"sep": frac(den, f32(dv + f32(1e-15)))}
    # addcdiv
    step = -(0.0025 / (1 - 0.9 ** 3))
    d = [p.cuda()]
    torch._foreach_addcdiv_(d, [m.cuda()], [torch.from_numpy(den).cuda()], [step])
    out = d[0].cpu().numpy()
    st = f32(step)
    P_ = p.numpy()
    q = f32(M / den)
    res["addcdiv"] = {"sep_s(m/d)": frac(out, f32(P_ + f32(st * q))), "fma_s(m/d)": frac(out, fma(st, q, P_)),
                      "sep_(sm)/d": frac(out, f32(P_ + f32(f32(st * M) / den)))}
    print(json.dumps(res))


if __name__ == "__main__":
    main()
