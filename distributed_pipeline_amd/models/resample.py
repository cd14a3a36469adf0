"""Timestep samplers for diffusion training (DiffuSeq ``resample.py`` semantics).

* ``uniform``    - t ~ U{0..T-1}, weights 1 (benchmark default).
* ``lossaware``  - loss-second-moment resampling: keep the last ``history``
  losses per t; once every t is warm sample p(t) ~ sqrt(E[L_t^2]) mixed with
  ``uniform_prob`` uniform mass and importance-weight 1/(T p(t)).  Local losses
  are gathered from all ranks with two all_gathers (sizes, padded values)
  (SURVEY X-8).
* ``fixstep``    - always t = T-1 (debugging).

Sampling runs on the device with ``torch.multinomial`` / ``randint`` (HIP-graph
safe); only ``update_with_local_losses`` touches the host.
"""
import numpy as np
import torch
import torch.distributed as dist


class ScheduleSampler:
    def __init__(self, num_timesteps):
        self.num_timesteps = num_timesteps

    def weights(self):
        raise NotImplementedError

    def sample(self, batch_size, device):
        w = self.weights()
        p = torch.as_tensor(w / np.sum(w), dtype=torch.float32, device=device)
        idx = torch.multinomial(p, batch_size, replacement=True)
        weights = 1.0 / (len(p) * p[idx])
        return idx, weights


class UniformSampler(ScheduleSampler):
    graph_safe = True  # device-side draw from the default CUDA generator (graph-capturable)

    def weights(self):
        return np.ones([self.num_timesteps])

    def sample(self, batch_size, device):
        t = torch.randint(0, self.num_timesteps, (batch_size,), device=device)
        return t, torch.ones(batch_size, dtype=torch.float32, device=device)


class FixSampler(ScheduleSampler):
    graph_safe = True

    def weights(self):
        w = np.zeros([self.num_timesteps])
        w[-1] = 1.0
        return w

    def sample(self, batch_size, device):
        t = torch.full((batch_size,), self.num_timesteps - 1, dtype=torch.long, device=device)
        return t, torch.ones(batch_size, dtype=torch.float32, device=device)


class LossSecondMomentResampler(ScheduleSampler):
    def __init__(self, num_timesteps, history_per_term=10, uniform_prob=0.001):
        super().__init__(num_timesteps)
        self.history_per_term = history_per_term
        self.uniform_prob = uniform_prob
        self._loss_history = np.zeros([num_timesteps, history_per_term], dtype=np.float64)
        self._loss_counts = np.zeros([num_timesteps], dtype=np.int64)

    def weights(self):
        if not self._warmed_up():
            return np.ones([self.num_timesteps], dtype=np.float64)
        w = np.sqrt(np.mean(self._loss_history ** 2, axis=-1))
        w /= np.sum(w)
        w *= 1 - self.uniform_prob
        w += self.uniform_prob / len(w)
        return w

    def update_with_local_losses(self, local_ts, local_losses):
        """Gather (t, loss) from every rank, then update the history."""
        if dist.is_available() and dist.is_initialized():
            dev = local_ts.device
            world = dist.get_world_size()
            n = torch.tensor([local_ts.numel()], dtype=torch.int64, device=dev)
            sizes = [torch.zeros_like(n) for _ in range(world)]
            dist.all_gather(sizes, n)
            max_n = int(max(s.item() for s in sizes))
            ts_pad = torch.zeros(max_n, dtype=torch.int64, device=dev)
            ls_pad = torch.zeros(max_n, dtype=torch.float32, device=dev)
            ts_pad[: local_ts.numel()] = local_ts.to(torch.int64)
            ls_pad[: local_losses.numel()] = local_losses.float()
            ts_all = [torch.zeros_like(ts_pad) for _ in range(world)]
            ls_all = [torch.zeros_like(ls_pad) for _ in range(world)]
            dist.all_gather(ts_all, ts_pad)
            dist.all_gather(ls_all, ls_pad)
            ts = [x.item() for y, s in zip(ts_all, sizes) for x in y[: int(s.item())]]
            ls = [x.item() for y, s in zip(ls_all, sizes) for x in y[: int(s.item())]]
        else:
            ts = local_ts.tolist()
            ls = local_losses.float().tolist()
        self.update_with_all_losses(ts, ls)

    def update_with_all_losses(self, ts, losses):
        for t, loss in zip(ts, losses):
            if self._loss_counts[t] == self.history_per_term:
                self._loss_history[t, :-1] = self._loss_history[t, 1:]
                self._loss_history[t, -1] = loss
            else:
                self._loss_history[t, self._loss_counts[t]] = loss
                self._loss_counts[t] += 1

    def _warmed_up(self):
        return (self._loss_counts == self.history_per_term).all()


def create_named_schedule_sampler(name, diffusion):
    if name == "uniform":
        return UniformSampler(diffusion.num_timesteps)
    if name == "lossaware":
        return LossSecondMomentResampler(diffusion.num_timesteps)
    if name == "fixstep":
        return FixSampler(diffusion.num_timesteps)
    raise NotImplementedError(f"unknown schedule sampler: {name}")
