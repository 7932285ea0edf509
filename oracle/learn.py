"""SAC / TD3 learn() restated in PyTorch-CPU fp32 — TEST INFRASTRUCTURE.

(see oracle/__init__.py).  Restates majidsina/rlmd:
  SAC  algos/algo_sac.py:300-367 (_multi_step_target), :369-595 (learn), :597-615 (Polyak)
       algos/networks_sac.py:101-178 (forward, stochastic_uv_gaussian), :180-220
       (stochastic_uv_laplace), :222-258 (stochastic_mv_gaussian), :346-362 (critic)
  TD3  algos/algo_td3.py:302-361, :363-531, :533-563; algos/networks_td3.py:76-91, :152-168
  losses tools/critic_loss.py:26-453 (per-sample losses, top-k, aggregator_fast, zipf_plot,
       cim_size, nagy_algo)
  Adam torch.optim.Adam defaults (the reference's optimiser), written out here.
Parameters live in one flat f32 tensor per role in the same layout as
librlmd_amd.so: trainable [actor | critic_1 | critic_2], targets alike.
Random draws (mini-batch, policy noise) are injected, as in the GPU parity hook.

precision="bf16" (the headline C2 arithmetic) restates the same update with
bf16 operands exactly where librlmd_amd's fused update rounds them (RNE; every
product of two bf16 values is exact in f32, sums stay f32):
  forward   h1 = relu(x W1^T + b1) in f32 -> bf16(h1) @ bf16(W2)^T (the fc2
            compute copy) + b2 -> relu -> heads in f32  (rows.hip mlp_rows:
            layer1 / mfma_rows / fwd_epilogue);
  critic    dW2 = (bf16(dq w3) [h2 > 0])^T bf16(h1); dW3 = dq . bf16(h2);
            dh1 = dq U1 with U1 = [h1 > 0] (bf16([h2 > 0] w3) @ bf16(W2)),
            dW1 = dh1^T x in f32  (update.hip critic_update_kernel, rows.hip basis_pass);
  actor     dq/da = ([e1 > 0] (bf16([e2 > 0] w3) @ bf16(W2))) W1[:, S:]  (qeval_rows);
            dh2 = [h2 > 0] (gh . W_heads) in f32, dW2 = bf16(dh2)^T bf16(h1),
            dW_heads = gh^T bf16(h2), dh1 = sum_h gh_h U_h with
            U_h = [h1 > 0] (bf16([h2 > 0] W_head[h]) @ bf16(W2))  (actor_update_kernel).
The gradients are then formed explicitly (autograd only through the loss and
the policy sampling, whose arithmetic is f32 on the device too); with the
rounding switched off the explicit form equals autograd (tests/test_oracle_learn.py).
path="chain" restates the launch chain instead (RLMD_NO_FUSED_UPDATE=1 /
RLMD_NO_FUSED_ACTOR=1, and every B > 512): dh1 = [h1 > 0] (bf16(dh2) @ bf16(W2))
(rows.hip cbwd_rows / abwd_rows), dL/da through bf16(dq w3 [h2 > 0]), and the
weight-gradient GEMM's bf16 operands: dW = bf16(G)^T bf16(X), db = sum bf16(G)
(gemm.hip GEMM_BWD_W, the bias as a ones column).
"""
import math

import numpy as np
import torch
import torch.nn.functional as F

LOSSES = ["MSE", "HUB", "MAE", "HSC", "CAU", "TCAU", "CIM", "MSE2", "MSE4", "MSE6"]


def net_layout(inp, h1, h2, out, heads):
    """[(name, shape)] in torch nn.Linear parameter order; heads = head layer names."""
    lay = [("fc1.weight", (h1, inp)), ("fc1.bias", (h1,)), ("fc2.weight", (h2, h1)), ("fc2.bias", (h2,))]
    for hd in heads:
        lay += [(hd + ".weight", (out, h2)), (hd + ".bias", (out,))]
    return lay


def layout(algo, S, A, h1, h2):
    """{net: [(name, shape, offset)]}, total size; nets actor, critic_1, critic_2."""
    nets = {"actor": net_layout(S, h1, h2, A, ("pi", "log_scale") if algo == "SAC" else ("mu",)),
            "critic_1": net_layout(S + A, h1, h2, 1, ("q_value",)),
            "critic_2": net_layout(S + A, h1, h2, 1, ("q_value",))}
    out, off = {}, 0
    for nm, lay in nets.items():
        out[nm] = []
        for pn, shp in lay:
            out[nm].append((pn, shp, off))
            off += int(np.prod(shp))
    return out, off


def views(flat, lay):
    return {nm: {pn: flat[o:o + int(np.prod(shp))].view(shp) for pn, shp, o in entries}
            for nm, entries in lay.items()}


def flatten(state_dicts, lay, total):
    """state_dicts: {net: {param_name: array}} -> flat f32 numpy."""
    out = np.zeros(total, dtype=np.float32)
    for nm, entries in lay.items():
        for pn, shp, o in entries:
            out[o:o + int(np.prod(shp))] = np.asarray(state_dicts[nm][pn], dtype=np.float32).ravel()
    return out


def mlp(p, x, head):
    h = F.relu(F.linear(x, p["fc1.weight"], p["fc1.bias"]))
    h = F.relu(F.linear(h, p["fc2.weight"], p["fc2.bias"]))
    return h, F.linear(h, p[head + ".weight"], p[head + ".bias"])


def rbf(x):
    """Round to bf16 (RNE, as the kernels' v_cvt / to_bf16) and back to f32."""
    return x.to(torch.bfloat16).to(torch.float32)


def ident(x):
    return x


def mlp_rows(p, x, heads, bf):
    """The row kernels' forward: (h1 f32, h2 f32, [head outputs incl. bias])."""
    h1 = F.relu(F.linear(x, p["fc1.weight"], p["fc1.bias"]))
    h2 = F.relu(bf(h1) @ bf(p["fc2.weight"]).T + p["fc2.bias"])
    return h1, h2, [h2 @ p[h + ".weight"].T + p[h + ".bias"] for h in heads]


def basis(h1, h2, w, W2, bf):
    """[h1 > 0] (bf16([h2 > 0] w) @ bf16(W2)): the backward basis of an output
    row vector w [H2] (rows.hip basis_pass / qeval_rows head jobs)."""
    return (h1 > 0).float() * (bf((h2 > 0).float() * w) @ bf(W2))


def zipf_axis(k):
    zx = (torch.ones(k) + k).view(-1)
    zx = zx / torch.arange(1, k + 1, dtype=torch.float32)
    zx = torch.log(zx)
    zx = zx - torch.mean(zx)
    return zx, torch.sum(zx**2)


def per_sample_loss(lt, est, tgt, scale, kernel):
    d = tgt - est
    if lt == "MSE":
        return d**2
    if lt in ("MSE2", "MSE4", "MSE6"):
        return d ** (2 + int(lt[3:]))
    if lt == "MAE":
        return torch.abs(d)
    if lt == "HUB":
        a = torch.abs(d)
        return torch.where(a < 1, 0.5 * a**2, a - 0.5)
    if lt == "HSC":
        return torch.sqrt(1 + d**2) - 1
    if lt in ("CAU", "TCAU"):
        return torch.log(1 + (d / scale) ** 2)
    if lt == "CIM":
        return 1 - torch.exp(-(d**2) / (2 * kernel**2)) / math.sqrt(2 * math.pi * kernel)
    raise ValueError(lt)


def truncate(x):
    """3-sigma rejection to zero (critic_loss.py:26-50)."""
    sigma, mean = torch.std_mean(x, unbiased=False)
    return torch.where(torch.abs(x - mean) > 3 * sigma, x - x, x)


def critic_losses(q1, q2, y, B, k, lt, scale, kern, zx, zx2, log_noise):
    """loss_function + aggregator_fast: (mean, min, max, alpha) per critic."""
    if lt == "TCAU":
        e1, t1 = truncate(q1), truncate(y)
        e2, t2 = truncate(q2), truncate(y)
    else:
        e1, t1, e2, t2 = q1, y, q2, y
    l1 = per_sample_loss(lt, e1, t1, scale[0], kern[0]).view(-1)
    l2 = per_sample_loss(lt, e2, t2, scale[1], kern[1]).view(-1)
    if B > k:
        order = torch.argsort((l1 + l2).detach(), descending=True, stable=True)[:k]
        l1, l2 = l1[order], l2[order]
    out = []
    for l in (l1, l2):
        ls = torch.sort(l.detach(), descending=True)[0]
        lg = torch.log(ls + log_noise)
        alpha = 1 / (torch.sum(zx * (lg - torch.mean(lg))) / zx2)
        out.append((torch.mean(l), torch.min(l), torch.max(l), alpha))
    return out


def cim_size(q, y):
    return torch.std(((y - q) ** 2).detach(), unbiased=False)


def nagy(q, y, scale):
    arg = ((y - q).detach() / scale) ** 2
    inv = 1 / torch.mean(1 / (1 + arg))
    return float(scale * torch.sqrt(inv - 1)) if inv > 1 else float(scale)


class Adam:
    """torch.optim.Adam(lr) single-tensor update (betas .9/.999, eps 1e-8)."""

    def __init__(self, n, lr):
        self.m = torch.zeros(n)
        self.v = torch.zeros(n)
        self.t = 0
        self.lr = lr

    def step(self, p, g):
        self.t += 1
        self.m.lerp_(g, 1 - 0.9)
        self.v.mul_(0.999).addcmul_(g, g, value=1 - 0.999)
        bc1 = 1 - 0.9**self.t
        bc2 = 1 - 0.999**self.t
        denom = (self.v.sqrt() / math.sqrt(bc2)).add_(1e-8)
        p.addcdiv_(self.m, denom, value=-self.lr / bc1)


class OracleLearner:
    def __init__(self, algo, S, A, h1, h2, B, k, loss_type, params, targets, *, gamma=0.99,
                 tau=5e-3, lr_actor=None, lr_critic=None, lr_temp=3e-4, reward_scale=1.0,
                 max_action=0.99, ls_min=-20.0, ls_max=2.0, reparam_noise=1e-6, log_noise=1e-6,
                 cauchy=1.0, logtemp=0.0, policy_noise=0.1, target_noise=0.2, target_clip=0.5,
                 actor_interval=None, target_critic_update=None, target_actor_update=2,
                 temp_interval=1, actor_topk=True, s_dist="N", precision="fp32", explicit=None, path="fused"):
        sac = algo == "SAC"
        # explicit gradients (the kernels' rounding points when bf16); fp32 keeps
        # autograd unless explicit=True (the CPU check that both forms agree)
        self.bf = rbf if precision == "bf16" else ident
        self.explicit = precision == "bf16" if explicit is None else explicit
        self.path = path
        self.s_dist = s_dist
        self.algo, self.S, self.A, self.B, self.k, self.lt = algo, S, A, B, k, loss_type
        self.lay, self.n = layout(algo, S, A, h1, h2)
        self.P = torch.tensor(params, dtype=torch.float32).clone()
        self.T = torch.tensor(targets, dtype=torch.float32).clone()
        self.gamma, self.tau, self.reward_scale, self.max_action = gamma, tau, reward_scale, max_action
        self.ls_min, self.ls_max, self.reparam_noise = ls_min, ls_max, reparam_noise
        self.log_noise = torch.tensor(log_noise)
        self.cauchy = [cauchy, cauchy]
        self.log_alpha = torch.tensor(float(logtemp))
        self.policy_noise = policy_noise * max_action
        self.target_noise = target_noise * max_action
        self.target_clip = target_clip * max_action
        self.actor_interval = actor_interval or (1 if sac else 2)
        self.target_critic_update = target_critic_update or (1 if sac else 2)
        self.target_actor_update = target_actor_update
        self.temp_interval = temp_interval
        self.actor_topk = actor_topk
        lr_a = lr_actor or (3e-4 if sac else 1e-3)
        lr_c = lr_critic or (3e-4 if sac else 1e-3)
        a0 = self.lay["actor"][0][2]
        c0 = self.lay["critic_1"][0][2]
        self.a_rng = (a0, c0)
        self.c_rng = (c0, self.n)
        self.opt_a = Adam(c0 - a0, lr_a)
        self.opt_c = Adam(self.n - c0, lr_c)
        self.opt_t = Adam(1, lr_temp)
        self.zx, self.zx2 = zipf_axis(k)
        self.cntr = 0

    def nets(self, flat):
        return views(flat, self.lay)

    def load_state(self, params, targets, adam_m, adam_v, cauchy, log_alpha):
        """Take another learner's state (flat tensors in this layout): the parity
        tests start each oracle update from the device's own state, so that a
        difference measures that update's arithmetic alone."""
        self.P = torch.as_tensor(params, dtype=torch.float32).clone()
        self.T = torch.as_tensor(targets, dtype=torch.float32).clone()
        m = torch.as_tensor(adam_m, dtype=torch.float32)
        v = torch.as_tensor(adam_v, dtype=torch.float32)
        for opt, (lo, hi) in ((self.opt_a, self.a_rng), (self.opt_c, self.c_rng)):
            opt.m, opt.v = m[lo:hi].clone(), v[lo:hi].clone()
        self.cauchy = [float(cauchy[0]), float(cauchy[1])]
        self.log_alpha = torch.tensor(float(log_alpha))

    def policy(self, p, s, eps, stochastic=True):
        """SAC stochastic_uv_gaussian / _uv_laplace / _mv_gaussian (s_dist N / L / MVN)
        or deterministic_policy; TD3 forward.  eps: the injected noise (Laplace: the
        uniform w of Laplace.rsample)."""
        h, mu = mlp(p, s, "pi" if self.algo == "SAC" else "mu")
        if self.algo == "TD3":
            return torch.tanh(mu) * self.max_action, None
        if not stochastic:
            return torch.tanh(mu) * self.max_action, None
        ls = F.linear(h, p["log_scale.weight"], p["log_scale.bias"])
        ls = torch.clamp(ls, self.ls_min, self.ls_max)
        scale = ls.exp()
        if self.s_dist == "L":  # torch Laplace: loc - scale sign(w) log1p(-|w|)
            u = mu - scale * eps.sign() * torch.log1p(-eps.abs())
            lp = (-torch.log(2 * scale) - torch.abs(u - mu) / scale).sum(1)
        elif self.s_dist == "MVN":  # scale used as the variance: L = cholesky(diag) = sqrt
            sd = torch.sqrt(scale)
            u = mu + sd * eps
            z = (u - mu) / sd
            lp = -0.5 * (self.A * math.log(2 * math.pi) + (z * z).sum(1)) - torch.log(sd).sum(1)
        else:
            u = mu + eps * scale
            lp = (-((u - mu) ** 2) / (2 * scale**2) - torch.log(scale) - math.log(math.sqrt(2 * math.pi))).sum(1)
        a = torch.tanh(u) * self.max_action
        lp = lp - torch.log(1 - (a / self.max_action) ** 2 + self.reparam_noise).sum(1)
        return a, lp

    def learn(self, s, a, r, s2, done, eps_a, eps_b=None, eff=None):
        """One learn() on an injected mini-batch; returns (loss[11], logtemp, loss_params[4])."""
        if self.explicit:
            return self.learn_explicit(s, a, r, s2, done, eps_a, eps_b, eff)
        sac = self.algo == "SAC"
        s, a, r, s2 = (torch.as_tensor(x, dtype=torch.float32) for x in (s, a, r, s2))
        done = torch.as_tensor(done, dtype=torch.bool)
        eff = torch.ones(self.B, dtype=torch.int32) if eff is None else torch.as_tensor(eff)
        eps_a = torch.as_tensor(eps_a, dtype=torch.float32)
        B, k = self.B, self.k
        with torch.no_grad():
            Pn, Tn = self.nets(self.P), self.nets(self.T)
            if sac:
                a2, lp2 = self.policy(Pn["actor"], s2, eps_a)
            else:
                noise = (eps_a * self.target_noise).clamp(-self.target_clip, self.target_clip)
                a2 = (mlp(Tn["actor"], s2, "mu")[1].tanh() * self.max_action + noise).clamp(
                    -self.max_action, self.max_action)
            x2 = torch.cat([s2, a2], 1)
            qt1 = mlp(Tn["critic_1"], x2, "q_value")[1].view(-1)
            qt2 = mlp(Tn["critic_2"], x2, "q_value")[1].view(-1)
            qt1[done], qt2[done] = 0.0, 0.0
            m = torch.min(qt1, qt2)
            g = self.gamma ** eff.to(torch.float32)
            if sac:
                y = self.reward_scale * r + g * m - self.log_alpha.exp() * lp2
            else:
                y = r + g * m
        y = y.view(B, 1)
        # critics
        P = self.P.clone().requires_grad_(True)
        Pn = self.nets(P)
        x = torch.cat([s, a], 1)
        q1 = mlp(Pn["critic_1"], x, "q_value")[1]
        q2 = mlp(Pn["critic_2"], x, "q_value")[1]
        kern = [float(cim_size(q1, y)), float(cim_size(q2, y))]
        (m1, mn1, mx1, al1), (m2, mn2, mx2, al2) = critic_losses(
            q1, q2, y, B, k, self.lt, self.cauchy, kern, self.zx, self.zx2, self.log_noise)
        closs = 0.5 * (m1 + m2) if sac else m1 + m2
        gP = torch.autograd.grad(closs, P)[0]
        c0, c1 = self.c_rng
        with torch.no_grad():
            self.opt_c.step(self.P[c0:c1], gP[c0:c1])
        self.cauchy = [nagy(q1, y, self.cauchy[0]), nagy(q2, y, self.cauchy[1])]
        self.cntr += 1
        if self.cntr % self.target_critic_update == 0:
            with torch.no_grad():
                self.T[c0:c1] = self.tau * self.P[c0:c1] + (1 - self.tau) * self.T[c0:c1]
        loss = [m1.item(), m2.item(), mn1.item(), mn2.item(), mx1.item(), mx2.item(), np.nan, np.nan,
                al1.item(), al2.item(), np.nan]
        logtemp = float(self.log_alpha) if sac else np.nan
        lp_out = [self.cauchy[0], self.cauchy[1], kern[0], kern[1]]
        if self.cntr % self.actor_interval != 0:
            return loss, logtemp, lp_out
        # actor
        P = self.P.clone().requires_grad_(True)
        Pn = self.nets(P)
        a0, a1 = self.a_rng
        if sac:
            an, lp = self.policy(Pn["actor"], s, torch.as_tensor(eps_b, dtype=torch.float32))
            xn = torch.cat([s, an], 1)
            qa = mlp(Pn["critic_1"], xn, "q_value")[1]
            qb = mlp(Pn["critic_2"], xn, "q_value")[1]
            v = (torch.min(qa, qb).view(-1) - self.log_alpha.exp() * lp).view(-1)
            if self.actor_topk:
                v = v.sort(descending=True)[0][:k]
        else:
            an = mlp(Pn["actor"], s, "mu")[1].tanh() * self.max_action
            v = mlp(Pn["critic_1"], torch.cat([s, an], 1), "q_value")[1].view(-1)
            if self.actor_topk:
                v = v.sort(descending=False)[0][:k]
        aloss = -torch.mean(v)
        gP = torch.autograd.grad(aloss, P)[0]
        with torch.no_grad():
            self.opt_a.step(self.P[a0:a1], gP[a0:a1])
        loss[-1] = aloss.item()
        if not sac:
            if self.cntr % self.target_actor_update == 0:
                with torch.no_grad():
                    self.T[a0:a1] = self.tau * self.P[a0:a1] + (1 - self.tau) * self.T[a0:a1]
            return loss, logtemp, lp_out
        if self.cntr % self.temp_interval == 0:
            la = self.log_alpha.clone().requires_grad_(True)
            tl = torch.mean(-(la.exp() * (lp.detach() + (-self.A))))
            gl = torch.autograd.grad(tl, la)[0]
            t = self.log_alpha.view(1).clone()
            self.opt_t.step(t, gl.view(1))
            self.log_alpha = t[0].clone()
            logtemp = float(self.log_alpha)
        return loss, logtemp, lp_out

    # ------------------------------------------------------------------
    # explicit-gradient form (bf16 rounding points of the fused update)
    # ------------------------------------------------------------------
    def sample_heads(self, mu, ls_raw, eps):
        """The policy sample from the heads' outputs (the f32 arithmetic after the
        heads: rlmd_policy.h / networks_sac.py:138-266): (a, logp)."""
        if self.algo == "TD3":
            return torch.tanh(mu) * self.max_action, None
        scale = torch.clamp(ls_raw, self.ls_min, self.ls_max).exp()
        if self.s_dist == "L":
            u = mu - scale * eps.sign() * torch.log1p(-eps.abs())
            lp = (-torch.log(2 * scale) - torch.abs(u - mu) / scale).sum(1)
        elif self.s_dist == "MVN":
            sd = torch.sqrt(scale)
            u = mu + sd * eps
            z = (u - mu) / sd
            lp = -0.5 * (self.A * math.log(2 * math.pi) + (z * z).sum(1)) - torch.log(sd).sum(1)
        else:
            u = mu + eps * scale
            lp = (-((u - mu) ** 2) / (2 * scale**2) - torch.log(scale) - math.log(math.sqrt(2 * math.pi))).sum(1)
        a = torch.tanh(u) * self.max_action
        lp = lp - torch.log(1 - (a / self.max_action) ** 2 + self.reparam_noise).sum(1)
        return a, lp

    def _grads_into(self, flat, net, grads):
        """Write {param name: gradient} of one net into the flat gradient buffer."""
        for pn, shp, o in self.lay[net]:
            flat[o:o + int(np.prod(shp))] = grads[pn].reshape(-1)

    def learn_explicit(self, s, a, r, s2, done, eps_a, eps_b=None, eff=None):
        sac = self.algo == "SAC"
        bf = self.bf
        s, a, r, s2 = (torch.as_tensor(x, dtype=torch.float32) for x in (s, a, r, s2))
        done = torch.as_tensor(done, dtype=torch.bool)
        eff = torch.ones(self.B, dtype=torch.int32) if eff is None else torch.as_tensor(eff)
        eps_a = torch.as_tensor(eps_a, dtype=torch.float32)
        B, k, S, A = self.B, self.k, self.S, self.A
        ah = ("pi", "log_scale") if sac else ("mu",)
        with torch.no_grad():
            Pn, Tn = self.nets(self.P), self.nets(self.T)
            # target path (fwd_rows jobs 0-1)
            if sac:
                _, _, hd = mlp_rows(Pn["actor"], s2, ah, bf)
                a2, lp2 = self.sample_heads(hd[0], hd[1], eps_a)
            else:
                _, _, hd = mlp_rows(Tn["actor"], s2, ah, bf)
                noise = (eps_a * self.target_noise).clamp(-self.target_clip, self.target_clip)
                a2 = (hd[0].tanh() * self.max_action + noise).clamp(-self.max_action, self.max_action)
            x2 = torch.cat([s2, a2], 1)
            qt1 = mlp_rows(Tn["critic_1"], x2, ("q_value",), bf)[2][0].view(-1)
            qt2 = mlp_rows(Tn["critic_2"], x2, ("q_value",), bf)[2][0].view(-1)
            qt1[done], qt2[done] = 0.0, 0.0
            m = torch.min(qt1, qt2)
            g = self.gamma ** eff.to(torch.float32)
            y = (self.reward_scale * r + g * m - self.log_alpha.exp() * lp2) if sac else r + g * m
            # online critics on (s, a) (fwd_rows jobs 2-3)
            x = torch.cat([s, a], 1)
            fw = [mlp_rows(Pn[c], x, ("q_value",), bf) for c in ("critic_1", "critic_2")]
        y = y.view(B, 1)
        q = [fw[i][2][0].clone().requires_grad_(True) for i in range(2)]
        kern = [float(cim_size(q[0].detach(), y)), float(cim_size(q[1].detach(), y))]
        (m1, mn1, mx1, al1), (m2, mn2, mx2, al2) = critic_losses(
            q[0], q[1], y, B, k, self.lt, self.cauchy, kern, self.zx, self.zx2, self.log_noise)
        closs = 0.5 * (m1 + m2) if sac else m1 + m2
        dq = [t.view(-1) for t in torch.autograd.grad(closs, q)]
        gP = torch.zeros_like(self.P)
        with torch.no_grad():
            for ci, cn in enumerate(("critic_1", "critic_2")):
                p = Pn[cn]
                h1, h2, _ = fw[ci]
                w3 = p["q_value.weight"][0]
                m2f = (h2 > 0).float()
                if self.path == "chain":  # cbwd_rows + the weight-gradient GEMM
                    dh2 = m2f * (dq[ci][:, None] * w3[None, :])
                    dh1 = (h1 > 0).float() * (bf(dh2) @ bf(p["fc2.weight"]))
                    gq = bf(dq[ci])
                    self._grads_into(gP, cn, {
                        "fc1.weight": bf(dh1).T @ bf(x), "fc1.bias": bf(dh1).sum(0),
                        "fc2.weight": bf(dh2).T @ bf(h1), "fc2.bias": bf(dh2).sum(0),
                        "q_value.weight": (gq @ bf(h2)).view(1, -1), "q_value.bias": gq.sum().view(1)})
                    continue
                a2g = bf(dq[ci][:, None] * w3[None, :]) * m2f  # update.hip form_a
                u1 = basis(h1, h2, w3, p["fc2.weight"], bf)
                g1 = dq[ci][:, None] * u1
                self._grads_into(gP, cn, {
                    "fc1.weight": g1.T @ x, "fc1.bias": g1.sum(0),
                    "fc2.weight": a2g.T @ bf(h1), "fc2.bias": w3 * (dq[ci][:, None] * m2f).sum(0),
                    "q_value.weight": (dq[ci] @ bf(h2)).view(1, -1), "q_value.bias": dq[ci].sum().view(1)})
            c0, c1 = self.c_rng
            self.opt_c.step(self.P[c0:c1], gP[c0:c1])
            # this update's gradients (nan: not stepped), for the tests' conditioning mask
            self.last_grad = torch.full_like(self.P, float("nan"))
            self.last_grad[c0:c1] = gP[c0:c1]
        self.cauchy = [nagy(q[0].detach(), y, self.cauchy[0]), nagy(q[1].detach(), y, self.cauchy[1])]
        self.cntr += 1
        if self.cntr % self.target_critic_update == 0:
            with torch.no_grad():
                self.T[c0:c1] = self.tau * self.P[c0:c1] + (1 - self.tau) * self.T[c0:c1]
        loss = [m1.item(), m2.item(), mn1.item(), mn2.item(), mx1.item(), mx2.item(), np.nan, np.nan,
                al1.item(), al2.item(), np.nan]
        logtemp = float(self.log_alpha) if sac else np.nan
        lp_out = [self.cauchy[0], self.cauchy[1], kern[0], kern[1]]
        if self.cntr % self.actor_interval != 0:
            return loss, logtemp, lp_out
        # ---- actor step: the policy on s (fwd_rows job 4, pre-step actor), the
        #      updated critics on (s, a_new) with dq/da (qeval_rows), the actor loss
        #      and its gradient (actor_update_kernel)
        a0, a1_ = self.a_rng
        with torch.no_grad():
            Pn = self.nets(self.P)
            pa = Pn["actor"]
            h1a, h2a, hd = mlp_rows(pa, s, ah, bf)
        mu = hd[0].clone().requires_grad_(True)
        lsr = hd[1].clone().requires_grad_(True) if sac else None
        eb = torch.as_tensor(eps_b, dtype=torch.float32) if sac else None
        an, lp = self.sample_heads(mu, lsr, eb)
        with torch.no_grad():
            xn = torch.cat([s, an.detach()], 1)
            qn, dqda, fwq = [], [], []
            for cn in (("critic_1", "critic_2") if sac else ("critic_1",)):
                p = Pn[cn]
                e1, e2, hq = mlp_rows(p, xn, ("q_value",), bf)
                qn.append(hq[0].view(-1))
                fwq.append((p, e1, e2))
                dqda.append(basis(e1, e2, p["q_value.weight"][0], p["fc2.weight"], bf) @ p["fc1.weight"][:, S:])
            alpha = self.log_alpha.exp()
            if sac:
                v = torch.min(qn[0], qn[1]) - alpha * lp.detach()
            else:
                v = qn[0]
            kk = min(B, k) if self.actor_topk else B
            # SAC descending, TD3 ascending; ties by row (the kernels' rank keys)
            order = torch.argsort(-v if sac else v, stable=True)[:kk] if self.actor_topk else torch.arange(B)
            sel = torch.zeros(B)
            sel[order] = 1.0
            aloss = -(v * sel).sum() / kk
            dv = -sel / kk
            if sac:
                g1 = torch.where(qn[0] < qn[1], 1.0, torch.where(qn[0] > qn[1], 0.0, 0.5))
                dqn = [dv * g1, dv * (1 - g1)]
                dlp = -alpha * dv
            else:
                dqn = [dv]
            if self.path == "chain":  # abwd_rows: dq scaled inside the bf16 operand
                da = sum((e1 > 0).float() * (bf((e2 > 0).float() * (d_[:, None] * p["q_value.weight"][0]))
                                             @ bf(p["fc2.weight"])) @ p["fc1.weight"][:, S:]
                         for d_, (p, e1, e2) in zip(dqn, fwq))
            else:
                da = sum(d_[:, None] * dd for d_, dd in zip(dqn, dqda))
        if sac:
            gmu, gls = torch.autograd.grad((da * an).sum() + (dlp * lp).sum(), [mu, lsr])
            gh = [gmu, gls]
        else:
            gh = [torch.autograd.grad((da * an).sum(), [mu])[0]]
        with torch.no_grad():
            wh = [pa[h + ".weight"] for h in ah]  # [A, H2] each
            m2a = (h2a > 0).float()
            dh2 = m2a * sum(g_ @ w_ for g_, w_ in zip(gh, wh))
            if self.path == "chain":  # abwd_rows dh1 + the weight-gradient GEMM
                dh1 = (h1a > 0).float() * (bf(dh2) @ bf(pa["fc2.weight"]))
                grads = {"fc1.weight": bf(dh1).T @ bf(s), "fc1.bias": bf(dh1).sum(0),
                         "fc2.weight": bf(dh2).T @ bf(h1a), "fc2.bias": bf(dh2).sum(0)}
                for h, g_ in zip(ah, gh):
                    grads[h + ".weight"] = bf(g_).T @ bf(h2a)
                    grads[h + ".bias"] = bf(g_).sum(0)
            else:
                dh1 = torch.zeros_like(h1a)
                for g_, w_ in zip(gh, wh):
                    for j in range(A):
                        dh1 += g_[:, j:j + 1] * basis(h1a, h2a, w_[j], pa["fc2.weight"], bf)
                grads = {"fc1.weight": dh1.T @ s, "fc1.bias": dh1.sum(0), "fc2.weight": bf(dh2).T @ bf(h1a),
                         "fc2.bias": dh2.sum(0)}
                for h, g_ in zip(ah, gh):
                    grads[h + ".weight"] = g_.T @ bf(h2a)
                    grads[h + ".bias"] = g_.sum(0)
            gP = torch.zeros_like(self.P)
            self._grads_into(gP, "actor", grads)
            self.last_grad[a0:a1_] = gP[a0:a1_]
            self.opt_a.step(self.P[a0:a1_], gP[a0:a1_])
        loss[-1] = aloss.item()
        if not sac:
            if self.cntr % self.target_actor_update == 0:
                with torch.no_grad():
                    self.T[a0:a1_] = self.tau * self.P[a0:a1_] + (1 - self.tau) * self.T[a0:a1_]
            return loss, logtemp, lp_out
        if self.cntr % self.temp_interval == 0:
            la = self.log_alpha.clone().requires_grad_(True)
            tl = torch.mean(-(la.exp() * (lp.detach() + (-self.A))))
            gl = torch.autograd.grad(tl, la)[0]
            t = self.log_alpha.view(1).clone()
            self.opt_t.step(t, gl.view(1))
            self.log_alpha = t[0].clone()
            logtemp = float(self.log_alpha)
        return loss, logtemp, lp_out
