"""Checkpoint loading and the autoregressive rollout driver.

* ``load_checkpoint`` follows MSFNO/Models/sfno/model.py:206-271 (``load_model``):
  optional ``"model_state"`` wrapper, the ``drop_vars`` filter, the DDP
  ``"module."`` prefix strip (and its ``"ged"`` entry), strict load first and
  ``strict=False`` on failure (the ECMWF weights lack the SHT buffers
  ``trans_down.weights`` / ``itrans_up.pct``).  Files are read with
  ``torch.load(weights_only=True)`` — nothing in a checkpoint is executed.
* ``Rollout`` is ``running()`` (model.py:289-372) without the GRIB I/O: the
  state stays on the GPU between 6 h steps (the reference copies every output
  to the host before writing it), ``normalise`` is model.py:273-279, and one
  step can be captured as a HIP graph and replayed.
"""
from __future__ import annotations

import warnings

import torch

DROP_VARS = ("module.norm.weight", "module.norm.bias")  # model.py:216


def load_checkpoint(model, checkpoint, map_location="cpu"):
    """Load a reference checkpoint (path or already-loaded dict) into ``model``.
    Returns ``(model, strict)`` where ``strict`` tells whether the strict load
    succeeded."""
    if isinstance(checkpoint, (str, bytes)) or hasattr(checkpoint, "read"):
        checkpoint = torch.load(checkpoint, map_location=map_location, weights_only=True)
    weights = checkpoint["model_state"] if "model_state" in checkpoint else checkpoint
    weights = {k: v for k, v in weights.items() if k not in DROP_VARS}
    if weights and next(iter(weights)).startswith("module."):
        weights = {k[7:]: v for k, v in weights.items() if k[7:] != "ged"}
    try:
        model.load_state_dict(weights)
        strict = True
    except RuntimeError as e:
        warnings.warn(f"loading state dict with strict=False ({str(e).splitlines()[0]})",
                      stacklevel=2)
        model.load_state_dict(weights, strict=False)
        strict = False
    model.eval()
    model.zero_grad()
    return model, strict


class Rollout:
    """On-device autoregressive stepping of a FourierNeuralOperatorNet[_Filmed].

    ``means`` / ``stds`` broadcast against the (B, C, H, W) state (the
    reference's global statistics, model.py:190-204).  ``film`` is the FiLM
    modulation passed to Filmed networks every step (or None)."""

    def __init__(self, model, means=None, stds=None, film=None, scale=1.0, graph=True):
        self.model = model
        self.means, self.stds = means, stds
        self.film, self.scale = film, scale
        self.use_graph = graph
        self._graph = None

    def normalise(self, data, reverse=False):
        """model.py:273-279."""
        if self.means is None:
            return data
        if reverse:
            return data * self.stds + self.means
        return (data - self.means) / self.stds

    def _step(self, x):
        if self.film is None:
            return self.model(x)
        return self.model(x, self.film, self.scale)

    def _capture(self, x):
        self._state = x.clone()
        self._step(self._state)  # warm-up: plans, descriptors, allocator pools
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            self._out = self._step(self._state)
        self._graph = g

    @torch.no_grad()
    def run(self, x0, steps, normalised_input=False):
        """Yields (step_index, denormalised output on the device) for ``steps``
        6 h steps starting from ``x0`` (raw fields unless ``normalised_input``)."""
        x = x0 if normalised_input else self.normalise(x0)
        x = x.contiguous()
        if self.use_graph and x.is_cuda:
            if self._graph is None or self._state.shape != x.shape:
                self._capture(x)
            self._state.copy_(x)
            for i in range(steps):
                self._graph.replay()
                # the graph's output buffer is overwritten by the next replay: hand the
                # caller a tensor of its own (normalise(reverse) already makes one)
                y = self.normalise(self._out, reverse=True)
                yield i, (y.clone() if y is self._out else y)
                self._state.copy_(self._out)
        else:
            for i in range(steps):
                x = self._step(x)
                yield i, self.normalise(x, reverse=True)
