"""Checkpoint loading and the autoregressive rollout driver.

* ``load_checkpoint`` follows MSFNO/Models/sfno/model.py:206-271 (``load_model``):
  optional ``"model_state"`` wrapper, the ``drop_vars`` filter, the DDP
  ``"module."`` prefix strip (and its ``"ged"`` entry), strict load first and
  ``strict=False`` on failure (the ECMWF weights lack the SHT buffers
  ``trans_down.weights`` / ``itrans_up.pct``).  Files are read with
  ``torch.load(weights_only=True)`` — nothing in a checkpoint is executed.
* ``load_filmed_checkpoint`` follows model.py:917-1033 (``FourCastNetv2_filmed.
  load_model``): the same SFNO load, the ``--retrain-film`` skip list, the
  FiLM-generator checkpoint merge (``"film_gen."`` prefix) and the freeze rule.
* ``Rollout`` is ``running()`` (model.py:289-372) without the GRIB I/O: the
  state stays on the GPU between 6 h steps (the reference copies every output
  to the host before writing it), ``normalise`` is model.py:273-279, and one
  step can be captured as a HIP graph and replayed.
"""
from __future__ import annotations

import warnings

import torch

DROP_VARS = ("module.norm.weight", "module.norm.bias")  # model.py:216


def _read(checkpoint, map_location):
    if isinstance(checkpoint, (str, bytes)) or hasattr(checkpoint, "read"):
        checkpoint = torch.load(checkpoint, map_location=map_location, weights_only=True)
    return checkpoint


def _load_with_fallback(module, weights, what="state dict"):
    """Strict load, then ``strict=False`` on a RuntimeError (model.py:240-256,
    956-964).  Returns whether the strict load succeeded."""
    try:
        module.load_state_dict(weights)
        return True
    except RuntimeError as e:
        warnings.warn(f"{what}: loading with strict=False ({str(e).splitlines()[0]})",
                      stacklevel=3)
        module.load_state_dict(weights, strict=False)
        return False


def _sfno_weights(checkpoint, skip=None):
    """model_state wrapper, drop_vars, the DDP "module." prefix and its "ged"
    entry (model.py:216-239, 927-955); ``skip(name)`` drops a key (the
    retrain_film rule, model.py:952 / 969)."""
    weights = checkpoint["model_state"] if "model_state" in checkpoint else checkpoint
    weights = {k: v for k, v in weights.items() if k not in DROP_VARS}
    prefixed = bool(weights) and next(iter(weights)).startswith("module.")
    out = {}
    for k, v in weights.items():
        name = k[7:] if prefixed else k
        if skip is not None and skip(name):
            continue
        if prefixed and name == "ged":
            continue
        out[name] = v
    return out


def load_checkpoint(model, checkpoint, map_location="cpu"):
    """Load a reference checkpoint (path or already-loaded dict) into ``model``
    (FourCastNetv2.load_model, model.py:207-271).  Returns ``(model, strict)``
    where ``strict`` tells whether the strict load succeeded."""
    weights = _sfno_weights(_read(checkpoint, map_location))
    strict = _load_with_fallback(model, weights)
    model.eval()
    model.zero_grad()
    return model, strict


def retrain_film_layers(film_layers):
    """The trainable-name substrings of ``--retrain-film`` (model.py:923): the FiLM
    generator, the decoder and the last ``film_layers`` blocks, counted down from
    block 11 as the reference writes it (a 12-block network)."""
    return ["film_gen", "decoder"] + ["blocks." + str(11 - i) for i in range(film_layers)]


def load_filmed_checkpoint(model, checkpoint, film_checkpoint=None, retrain_film=False,
                           film_layers=1, resume_checkpoint=None, map_location="cpu"):
    """FourCastNetv2_filmed.load_model (model.py:917-1033) for a
    FourierNeuralOperatorNet_Filmed:

    * SFNO weights as ``load_checkpoint``; with ``retrain_film`` (and no
      ``resume_checkpoint``) every key containing one of
      ``retrain_film_layers(film_layers)`` is skipped (model.py:952, 969), so
      those layers keep their fresh initialisation;
    * the FiLM-generator checkpoint's ``model_state`` is prefixed with
      ``"film_gen."`` unless it already is, and loaded into ``model.film_gen``
      (model.py:983-1003); if that load fails the reference retries with the raw
      checkpoint dict and ``strict=False``, which loads nothing: reproduced, with a
      warning;
    * freeze (model.py:1016-1023): with ``retrain_film`` every parameter outside
      those layers gets ``requires_grad=False``; otherwise every parameter whose
      name lacks ``"film_gen"``.

    Returns ``(model, strict)`` for the SFNO load."""
    model.zero_grad()
    grad_layers = retrain_film_layers(film_layers) if retrain_film else None

    def skip(name):
        return (retrain_film and resume_checkpoint is None
                and any(layer in name for layer in grad_layers))

    weights = _sfno_weights(_read(checkpoint, map_location), skip)
    strict = _load_with_fallback(model, weights, "SFNO weights")
    if film_checkpoint is not None:
        ck = _read(film_checkpoint, map_location)
        film_weights = ck["model_state"]
        if not next(iter(film_weights)).startswith("film_gen."):
            film_weights = {"film_gen." + k: v for k, v in film_weights.items()}
        if model.film_gen is None:
            raise ValueError("a FiLM-generator checkpoint needs model.film_gen")
        try:
            model.film_gen.load_state_dict(film_weights)
        except RuntimeError as e:
            warnings.warn("Film Gen: loading with strict=False, as the reference does "
                          f"(model.py:1003; nothing is loaded): {str(e).splitlines()[0]}",
                          stacklevel=2)
            model.film_gen.load_state_dict({k: v for k, v in ck.items()
                                            if isinstance(v, torch.Tensor)}, strict=False)
    for name, param in model.named_parameters():
        if retrain_film:
            if not any(layer in name for layer in grad_layers):
                param.requires_grad = False
        elif "film_gen" not in name:
            param.requires_grad = False
    model.eval()
    model.zero_grad()
    return model, strict


class Rollout:
    """On-device autoregressive stepping of a FourierNeuralOperatorNet[_Filmed], or
    of one rank's ``LatBandNet`` (the multi-GPU form of config 5: every rank steps
    its own latitude rows; x0 is then ``shard.take(x0)`` and the outputs are the
    rank's rows).

    ``means`` / ``stds`` broadcast against the (B, C, H, W) state (the
    reference's global statistics, model.py:190-204: per channel, so they apply to
    a rank's rows unchanged).  ``film`` is the FiLM modulation passed to Filmed
    networks every step (or None).  A sharded network with more than one rank is
    captured too when its exchanges run on RCCL (a ``TorchComm`` over the nccl
    backend: the collectives are recorded into the graph, model.py:327-331's
    per-step cost without the host launches); over gloo (host collectives) it steps
    eagerly, and a capture that fails on any rank makes every rank step eagerly
    (``TorchComm.all_agree``)."""

    def __init__(self, model, means=None, stds=None, film=None, scale=1.0, graph=True):
        self.model = model
        self.means, self.stds = means, stds
        self.film, self.scale = film, scale
        comm = getattr(model, "comm", None)
        device_comm = comm is not None and not getattr(comm, "host", True)
        # capture-or-eager must be one decision for all ranks (all_agree); a multi-rank
        # comm that cannot agree steps eagerly on every rank
        agreeable = device_comm and callable(getattr(comm, "all_agree", None))
        self.use_graph = graph and (getattr(model, "world", 1) == 1 or agreeable)
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
        quiesce = getattr(getattr(self.model, "comm", None), "quiesce", None)
        if callable(quiesce):
            quiesce()  # no RCCL work of the warm-up left for the watchdog to poll
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
        if self.use_graph and x.is_cuda and (self._graph is None or self._state.shape != x.shape):
            if getattr(self.model, "world", 1) == 1:
                self._capture(x)
            else:
                # capture-or-eager is decided by all ranks together: a rank whose
                # capture failed (a collective the backend cannot record) must not step
                # eagerly while its peers replay recorded collectives
                ok = True
                try:
                    self._capture(x)
                except RuntimeError:
                    ok = False
                    torch.cuda.synchronize()
                ok = self.model.comm.all_agree(ok)
                if not ok:
                    self._graph = None
                    self.use_graph = False
        if self.use_graph and x.is_cuda:
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
