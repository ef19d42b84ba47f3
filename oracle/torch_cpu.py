"""torch-CPU restatement of models/deepfm_pipeline.py — TEST / BASELINE INFRASTRUCTURE ONLY.

The CPU baseline BASELINE.md §2 plans: the reference's own TF-CPU path cannot run here
(TensorFlow 1.x is absent), so bench.py's `cpu_baseline` times this restatement of the same
graph on the host cores with torch's intra-op thread pool (all cores).  It follows the
numpy oracle (oracle/ctr_ref.py) op for op and is checked against it in
tests/test_oracle.py::test_torch_cpu_restatement_matches_numpy_oracle:

  tables        feats_emb [C+N, E], fm_first_order_emb [C+N, 1]     deepfm_pipeline.py:77-81
  row-0 zero    concat([zeros, V[1:]]) every step (dense gradient)   :83-86
  FM            idx = [cont 0..C-1 | cate + C], first = w1[idx]*val,
                second = 0.5((sum e)^2 - sum e^2)                    :89-110
  deep          x = [cont | V[cate] (raw ids)], relu(x W + b) x3      :117-153
  head          z = [first | second | deep] W_out + b, p = sigmoid   :155-173
  loss          tf.losses.log_loss(y, p) (eps 1e-7) + l2/2 |W_out|^2  :179-183
  optimizer     TF1 ApplyAdam over every trainable, dense            :184-188

The backward is torch autograd; the optimizer is TF1's dense ApplyAdam written as in-place
multi-threaded torch ops (m += (g - m)(1 - b1); v += (g^2 - v)(1 - b2);
p -= m alpha / (sqrt(v) + eps), alpha = lr sqrt(1 - b2^t) / (1 - b1^t)).
Only tests/ and bench.py's cpu_baseline leg import this module.
"""
import torch


class DeepFMPipelineCPU:
    """fm=False: models/dnn_pipeline.py (BASELINE C1) — the same deep input [cont | V[cate]] over
    the row-0-zeroed table (dnn_pipeline.py:68-107), no FM terms, the `deep_res` output layer
    with L2 on it (:114-131)."""

    def __init__(self, C, S, E, cate_index_size, hidden, P, lr=0.001, l2=1e-5, beta1=0.9, beta2=0.999,
                 eps=1e-8, logloss_eps=1e-7, fm=True):
        self.fm = fm
        self.C, self.S, self.E, self.hidden = C, S, E, list(hidden)
        self.lr, self.l2, self.b1, self.b2, self.eps, self.leps = lr, l2, beta1, beta2, eps, logloss_eps
        t = lambda a: torch.from_numpy(a.copy()).float().requires_grad_(True)
        self.params = {k: t(v) for k, v in P.items()}
        self.m = {k: torch.zeros_like(v) for k, v in self.params.items()}
        self.v = {k: torch.zeros_like(v) for k, v in self.params.items()}
        self.b1p = torch.tensor(beta1, dtype=torch.float32)
        self.b2p = torch.tensor(beta2, dtype=torch.float32)
        self.cidx = None

    def forward(self, batch):
        P, C, S, E = self.params, self.C, self.S, self.E
        cont = torch.from_numpy(batch["cont_feats"]).float()
        cate = torch.from_numpy(batch["cate_feats"]).long()
        lab = torch.from_numpy(batch["label"]).float().reshape(-1)
        B = lab.shape[0]
        V = torch.cat([torch.zeros(1, E), P["feats_emb"][1:]], 0)                     # :83-84
        if not self.fm:                                                              # dnn_pipeline.py
            h = torch.cat([cont, V[cate].reshape(B, S * E)], 1)
            for i in range(len(self.hidden)):
                h = torch.relu(h @ P["deep_%d" % i] + P["deep_bias_%d" % i])
            z = (h @ P["deep_res"])[:, 0] + P["deep_res_bias"][0, 0]                  # :119
            p = torch.sigmoid(z)
            loss = (-lab * torch.log(p + self.leps) - (1 - lab) * torch.log(1 - p + self.leps)).mean()
            return z, loss + self.l2 * 0.5 * (P["deep_res"] ** 2).sum()              # :131
        w1 = torch.cat([torch.zeros(1, 1), P["fm_first_order_emb"][1:]], 0)          # :85-86
        if self.cidx is None or self.cidx.shape[0] != B:
            self.cidx = torch.arange(C, dtype=torch.long).repeat(B, 1)               # :58-61
        idx = torch.cat([self.cidx, cate + C], 1)                                    # :89-90
        val = torch.cat([cont, torch.ones(B, S)], 1)                                 # :91
        first = w1[idx][:, :, 0] * val                                               # :95-97
        e = V[idx] * val[:, :, None]                                                 # :102-104
        s = e.sum(1)
        second = 0.5 * (s * s - (e * e).sum(1))                                      # :105-109
        h = torch.cat([cont, V[cate].reshape(B, S * E)], 1)                          # :120-123
        for i in range(len(self.hidden)):
            h = torch.relu(h @ P["deep_%d" % i] + P["deep_bias_%d" % i])             # :149-153
        feats = torch.cat([first, second, h], 1)                                     # :157
        z = (feats @ P["deep_fm_weight"])[:, 0] + P["deep_fm_bias"][0]               # :171
        p = torch.sigmoid(z)                                                         # :173
        loss = (-lab * torch.log(p + self.leps) - (1 - lab) * torch.log(1 - p + self.leps)).mean()   # :179
        loss = loss + self.l2 * 0.5 * (P["deep_fm_weight"] ** 2).sum()               # :183
        return z, loss

    @torch.no_grad()
    def _adam(self):
        one = torch.tensor(1.0)
        alpha = float(self.lr * torch.sqrt(one - self.b2p) / (one - self.b1p))
        omb1, omb2 = 1.0 - self.b1, 1.0 - self.b2
        for k, p in self.params.items():
            g, m, v = p.grad, self.m[k], self.v[k]
            m.add_((g - m).mul_(omb1))
            v.add_((g * g).sub_(v).mul_(omb2))
            p.sub_((m * alpha).div_(v.sqrt().add_(self.eps)))
            p.grad = None
        self.b1p = self.b1p * self.b1
        self.b2p = self.b2p * self.b2

    def train_step(self, batch):
        z, loss = self.forward(batch)
        loss.backward()
        self._adam()
        return z.detach(), float(loss.detach())
