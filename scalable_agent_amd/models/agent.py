"""IMPALA agent: conv torso -> LSTM-256 core -> policy/baseline heads.

Behaviour parity with the reference `Agent` (experiment.py:109-237):
  * torso (experiment.py:148-198): uint8 frame / 255, conv stack, ReLU,
    flatten, Linear(256), ReLU, concat [torso, clip(reward,-1,1),
    one_hot(last_action), instruction_encoding];
      - 'shallow' (active in the reference, :178-183): 32x8x8/4, 64x4x4/2,
        128x3x3/2, all TF-SAME;
      - 'deep' (IMPALA ResNet, commented out at :156-176, required by the north
        star): 3 stages of conv3x3 -> maxpool3x3/2 SAME -> 2 x residual block;
  * instruction encoder (:123-146): hashed words -> Embed(1000,20) ->
    LSTM(64) -> last valid output (zeros for an empty instruction);
  * core (:118, :228-235): LSTMBlockCell(256), state reset to zero *before*
    the step whenever done[t] is set;
  * heads (:200-210): Linear(A) logits, Linear(1) baseline, multinomial sample.

The module is backend-switchable: `backend='torch'` is the pure-PyTorch oracle
(CPU or GPU), `backend='hip'` routes every hot op through the hand-written
CDNA4 kernels in `scalable_agent_amd.ops` (fails loudly if they are missing).
Parameters are fp32 master weights in TF layouts (see models/layers.py).
"""

import math

import os

import torch
import torch.nn as nn
import torch.nn.functional as F

from ..structs import AgentOutput
from . import layers
from ..utils.knobs import measure_env

CORE_SIZE = 256
INSTR_BUCKETS = 1000
INSTR_EMBED = 20
INSTR_LSTM = 64


def _bf16_torso_ready(agent):
  """The fused bf16 torso kernels (conv_torso.hip) apply: bf16 compute and a
  shape they cover."""
  from ..ops import conv
  return (agent.compute_dtype == torch.bfloat16 and conv.TORSO_READY and
          conv.supports(agent))


def _hip_torso_ready(agent):
  """Some HIP torso covers the agent: the fused bf16 kernels, else the
  exact-fp32 kernels (any torso, C <= 4 frames)."""
  from ..ops import conv_f32
  return _bf16_torso_ready(agent) or conv_f32.supports(agent)


def torso_precision(agent):
  """'bf16' / 'fp32' (HIP kernels) or 'torch' for the torso that runs."""
  if agent.backend != 'hip':
    return 'torch'
  return 'bf16' if _bf16_torso_ready(agent) else 'fp32'


def hip_ops_in_use(agent):
  """Names of the ops this agent runs on hand-written HIP kernels."""
  if agent.backend != 'hip':
    return []
  ops = ['lstm_recurrence', 'vtrace_loss', 'rmsprop']
  if _hip_torso_ready(agent):
    ops += ['conv_torso_' + torso_precision(agent)]
  return ops


def torso_spec(torso, frame_shape):
  """Returns (conv layer specs, flattened feature size).

  Each spec: dict(kind='conv'|'pool'|'res', ...). Used by both backends.
  """
  h, w, c = frame_shape
  specs = []
  if torso == 'shallow':
    for i, (ch, k, s) in enumerate([(32, 8, 4), (64, 4, 2), (128, 3, 2)]):
      name = 'conv_2d' if i == 0 else 'conv_2d_%d' % i
      specs.append(dict(kind='conv', name=name, cin=c, cout=ch, k=k, s=s,
                        relu_out=True))
      h, w, c = layers.same_out(h, s), layers.same_out(w, s), ch
  elif torso == 'deep':
    n_conv = 0
    for i, (ch, nblocks) in enumerate([(16, 2), (32, 2), (32, 2)]):
      name = 'conv_2d' if n_conv == 0 else 'conv_2d_%d' % n_conv
      n_conv += 1
      specs.append(dict(kind='conv', name=name, cin=c, cout=ch, k=3, s=1,
                        relu_out=False))
      specs.append(dict(kind='pool'))
      h, w, c = layers.same_out(h, 2), layers.same_out(w, 2), ch
      for j in range(nblocks):
        specs.append(dict(kind='res', name='residual_%d_%d' % (i, j), ch=ch))
  else:
    raise ValueError('unknown torso %r' % torso)
  return specs, h * w * c, (h, w, c)


def _chunk_bounds(T, chunks, split=None):
  """Time-chunk boundaries [0, ..., T]: `chunks` equal chunks, or chunk
  lengths in the proportions of `split` ("9,9,2"), every chunk >= 1 step."""
  if split:
    w = [float(x) for x in split.split(',') if x.strip()]
    w = [max(x, 0.0) for x in w][:T] or [1.0]
    tot = sum(w) or 1.0
    b = [0]
    acc = 0.0
    for x in w[:-1]:
      acc += x
      b.append(min(T - (len(w) - len(b)), max(b[-1] + 1, int(round(T * acc / tot)))))
    b.append(T)
    return b
  chunks = max(1, min(int(chunks), T))  # no empty chunk when T < chunks
  return [(T * k) // chunks for k in range(chunks + 1)]


class Agent(nn.Module):
  """IMPALA agent (see module docstring)."""

  def __init__(self, num_actions, torso='shallow', frame_shape=(72, 96, 3),
               seed=None, backend='torch', compute_dtype=torch.float32,
               num_value_heads=1, pipeline_chunks=1):
    super().__init__()
    # > 1 (HIP backend on a GPU): the learner unroll is split into this many
    # time chunks; chunk k's LSTM recurrence runs on a side stream while the
    # conv torso of chunk k+1 runs on the main stream (see _pipelined_core).
    self.pipeline_chunks = int(pipeline_chunks)
    self._core_streams = {}
    # data-parallel learner: when a list, conv_features hands the core a
    # detached leaf and records (features, leaf) so the torso backward can
    # run as a separate phase (learner.Learner, gradient all-reduce overlap)
    self._split_torso = None
    self.num_actions = num_actions
    # > 1: one (PopArt-normalised) value output per task (popart.py)
    self.num_value_heads = int(num_value_heads)
    self.torso_kind = torso
    self.frame_shape = tuple(frame_shape)
    self.backend = backend
    self.compute_dtype = compute_dtype
    gen = None
    if seed is not None:
      gen = torch.Generator().manual_seed(int(seed))

    self.specs, flat, self.conv_out_shape = torso_spec(torso, self.frame_shape)
    self.flat_size = flat
    self.convnet = nn.ParameterDict()
    for sp in self.specs:
      if sp['kind'] == 'conv':
        w = nn.Parameter(torch.empty(sp['k'], sp['k'], sp['cin'], sp['cout']))
        layers.sonnet_linear_init_(w.data, gen)
        self.convnet[sp['name'] + '__w'] = w
        self.convnet[sp['name'] + '__b'] = nn.Parameter(torch.zeros(sp['cout']))
      elif sp['kind'] == 'res':
        for sub in ('conv_2d', 'conv_2d_1'):
          w = nn.Parameter(torch.empty(3, 3, sp['ch'], sp['ch']))
          layers.sonnet_linear_init_(w.data, gen)
          self.convnet[sp['name'] + '__' + sub + '__w'] = w
          self.convnet[sp['name'] + '__' + sub + '__b'] = nn.Parameter(
              torch.zeros(sp['ch']))

    self.linear_w = nn.Parameter(
        layers.sonnet_linear_init_(torch.empty(flat, CORE_SIZE), gen))
    self.linear_b = nn.Parameter(torch.zeros(CORE_SIZE))

    self.embed = nn.Parameter(
        layers.truncated_normal_(torch.empty(INSTR_BUCKETS, INSTR_EMBED),
                                 1.0, gen))
    self.language_lstm_kernel = nn.Parameter(layers.glorot_uniform_(
        torch.empty(INSTR_EMBED + INSTR_LSTM, 4 * INSTR_LSTM), gen))
    self.language_lstm_bias = nn.Parameter(torch.zeros(4 * INSTR_LSTM))

    self.core_input_size = CORE_SIZE + 1 + num_actions + INSTR_LSTM
    self.lstm_kernel = nn.Parameter(layers.glorot_uniform_(
        torch.empty(self.core_input_size + CORE_SIZE, 4 * CORE_SIZE), gen))
    self.lstm_bias = nn.Parameter(torch.zeros(4 * CORE_SIZE))

    self.policy_w = nn.Parameter(
        layers.sonnet_linear_init_(torch.empty(CORE_SIZE, num_actions), gen))
    self.policy_b = nn.Parameter(torch.zeros(num_actions))
    self.baseline_w = nn.Parameter(layers.sonnet_linear_init_(
        torch.empty(CORE_SIZE, self.num_value_heads), gen))
    self.baseline_b = nn.Parameter(torch.zeros(self.num_value_heads))

  # ------------------------------------------------------------------ naming
  def tf_variable_names(self):
    """Maps parameter names to reference-style TF variable names (§7.4)."""
    out = {}
    for name, _ in self.named_parameters():
      if name.startswith('convnet.'):
        tf = 'agent/convnet/' + name[len('convnet.'):].replace('__', '/')
      else:
        tf = {
            'linear_w': 'agent/linear/w', 'linear_b': 'agent/linear/b',
            'embed': 'agent/embed/embeddings',
            'language_lstm_kernel': 'agent/language_lstm/kernel',
            'language_lstm_bias': 'agent/language_lstm/bias',
            'lstm_kernel': 'agent/lstm_cell/kernel',
            'lstm_bias': 'agent/lstm_cell/bias',
            'policy_w': 'agent/policy_logits/w',
            'policy_b': 'agent/policy_logits/b',
            'baseline_w': 'agent/baseline/w',
            'baseline_b': 'agent/baseline/b'}[name]
      out[name] = tf
    return out

  def initial_state(self, batch_size, device=None):
    device = device or self.lstm_bias.device
    z = torch.zeros(batch_size, CORE_SIZE, device=device,
                    dtype=self.lstm_bias.dtype)
    return (z, z.clone())

  # ------------------------------------------------------------------ torso
  def _conv_params(self, name):
    return self.convnet[name + '__w'], self.convnet[name + '__b']

  def conv_features(self, frames):
    """frames uint8 [N,H,W,C] -> flattened conv features [N, flat]."""
    feats = self._conv_features(frames)
    split = self._split_torso
    if split is not None and feats.requires_grad:
      leaf = feats.detach().requires_grad_()
      split.append((feats, leaf))
      return leaf
    return feats

  def _conv_features(self, frames):
    if self.backend == 'hip' and frames.is_cuda:
      from .. import ops
      if _bf16_torso_ready(self):
        return ops.torso_forward(self, frames)
      # exact fp32 kernels (also for a bf16 agent whose shape the bf16
      # kernels do not cover); unsupported shapes raise, never fall back
      return ops.torso_forward_f32(self, frames)
    cdt = self.compute_dtype
    # float64: the learner-parity oracle (tests); else x/255 in fp32
    wide = torch.float64 if cdt == torch.float64 else torch.float32
    x = frames.to(wide) / 255.0
    if cdt != wide:
      x = x.to(cdt)
    for sp in self.specs:
      if sp['kind'] == 'conv':
        w, b = self._conv_params(sp['name'])
        x = layers.conv2d_same_nhwc(x, w.to(x.dtype), b.to(x.dtype), sp['s'])
        if sp['relu_out']:
          x = F.relu(x)
      elif sp['kind'] == 'pool':
        x = layers.maxpool_same_nhwc(x, 3, 2)
      else:
        block_in = x
        for sub in ('conv_2d', 'conv_2d_1'):
          w, b = self._conv_params(sp['name'] + '__' + sub)
          x = F.relu(x)
          x = layers.conv2d_same_nhwc(x, w.to(x.dtype), b.to(x.dtype), 1)
        x = x + block_in
    x = F.relu(x)
    return x.reshape(x.shape[0], -1)

  def torso_fc(self, feats):
    if self.backend == 'hip' and feats.is_cuda:
      from .. import ops
      if feats.dtype == torch.bfloat16:
        return ops.linear_relu(feats, self.linear_w, self.linear_b)
      return ops.linear_relu_f32(feats, self.linear_w, self.linear_b)
    w = self.linear_w.to(feats.dtype)
    b = self.linear_b.to(feats.dtype)
    out = F.relu(feats @ w + b)
    return out.float() if out.dtype == torch.bfloat16 else out

  def instruction_encoding(self, instr, n, device):
    """instr: None or (ids [N,L] int64, lengths [N] int64) -> [N, 64]."""
    if instr is None:
      return torch.zeros(n, INSTR_LSTM, device=device, dtype=self.embed.dtype)
    ids, lengths = instr
    ids = ids.reshape(n, -1).to(device)
    lengths = lengths.reshape(n).to(device)
    if self.backend == 'hip' and lengths.is_cuda:
      # embedding gather + the whole word loop + last-valid-word output in
      # one fused HIP kernel per direction (ops/lang.py); graph-safe (no
      # data-dependent host decisions)
      from .. import ops
      return ops.language_lstm(ids, lengths, self.embed,
                               self.language_lstm_kernel,
                               self.language_lstm_bias)
    capturing = lengths.is_cuda and torch.cuda.is_current_stream_capturing()
    if lengths.numel() == 0 or (not capturing and int(lengths.max()) == 0):
      return torch.zeros(n, INSTR_LSTM, device=device, dtype=self.embed.dtype)
    emb = layers.embedding_lookup(ids, self.embed)  # [N, L, 20]
    if self.backend == 'hip' and emb.is_cuda:
      # words are the time axis of the fused H=64 LSTM step kernels (K7
      # shares K9's kernels); the output is h at the last valid word
      from .. import ops
      z = torch.zeros(n, INSTR_LSTM, device=device)
      done = torch.zeros(ids.shape[1], n, dtype=torch.bool, device=device)
      hs, _ = ops.lstm_unroll(emb.transpose(0, 1).contiguous(), done, (z, z),
                              self.language_lstm_kernel,
                              self.language_lstm_bias,
                              exact=self.compute_dtype == torch.float32)
      last = (lengths - 1).clamp(min=0).view(1, n, 1).expand(1, n, INSTR_LSTM)
      out = hs.gather(0, last).squeeze(0)
      return out * (lengths > 0).unsqueeze(-1).to(out.dtype)
    c = torch.zeros(n, INSTR_LSTM, device=device, dtype=self.embed.dtype)
    h = torch.zeros_like(c)
    out = torch.zeros_like(c)
    for t in range(ids.shape[1]):
      h, c = layers.lstm_block_cell(emb[:, t], c, h, self.language_lstm_kernel,
                                    self.language_lstm_bias)
      out = torch.where((lengths - 1 == t).unsqueeze(-1), h, out)
    return out

  def core_inputs(self, frames, rewards, last_actions, instr):
    """Builds the LSTM core input [N, 256+1+A+64] (experiment.py:185-198)."""
    n = frames.shape[0]
    feats = self.conv_features(frames)
    torso_out = self.torso_fc(feats)
    dt = torso_out.dtype
    clipped_reward = torch.clamp(rewards.reshape(n, 1).to(dt), -1, 1)
    # tf.one_hot semantics: an out-of-range index gives a zero row (a
    # comparison, never a scatter - no out-of-bounds write under graphs)
    one_hot = (last_actions.reshape(n, 1).long() == torch.arange(
        self.num_actions, device=last_actions.device)).to(dt)
    instr_out = self.instruction_encoding(instr, n, frames.device)
    return torch.cat([torso_out, clipped_reward, one_hot, instr_out], dim=1)

  # ------------------------------------------------------------------ core
  def core_unroll(self, x, done, state):
    """x [T,B,F], done [T,B] bool, state (c,h) -> (h_all [T,B,256], state)."""
    if self.backend == 'hip':
      from .. import ops
      return ops.lstm_unroll(x, done, state, self.lstm_kernel, self.lstm_bias,
                             exact=self.compute_dtype == torch.float32)
    c, h = state
    T = x.shape[0]
    kx = self.lstm_kernel[:self.core_input_size]
    kh = self.lstm_kernel[self.core_input_size:]
    xw = torch.matmul(x, kx) + self.lstm_bias  # one GEMM for all steps
    outs = []
    for t in range(T):
      keep = (~done[t]).to(c.dtype).unsqueeze(-1)
      c = c * keep
      h = h * keep
      gates = xw[t] + h @ kh
      i, ci, f, o = gates.chunk(4, dim=-1)
      c = torch.tanh(ci) * torch.sigmoid(i) + c * torch.sigmoid(f + 1.0)
      h = torch.tanh(c) * torch.sigmoid(o)
      outs.append(h)
    return torch.stack(outs), (c, h)

  def _core_stream(self, device):
    s = self._core_streams.get(device)
    if s is None:
      s = torch.cuda.Stream(device)
      self._core_streams[device] = s
    return s

  def _pipelined_core(self, frames, reward, actions, instr, done, state,
                      chunks):
    """Time-chunked torso || LSTM pipeline (HIP backend, GPU only).

    The conv torso of time chunk k runs on the current (main) stream; the
    core of chunk k (fused torso-FC / core-input / x-projection GEMMs and
    the recurrence, ops.core_lstm - the same kernels as the unchunked path,
    with the LSTM state carried from chunk to chunk) runs on a side stream as
    soon as chunk k's features exist, overlapping the torso of chunk k+1.
    Autograd runs every backward node on its forward stream, so the backward
    overlaps the same way in reverse: once the recurrence of the last chunk
    has produced its input gradient, that chunk's torso backward runs while
    the recurrence backward continues on earlier chunks.  Both directions
    are fork/join DAGs that a captured hipGraph replays concurrently
    (tools/micro/graph_fork.hip).  The persistent conv grids leave
    cf32_cu_reserve() CUs per XCD to the side stream (set before capture).

    Chunk lengths: equal, or in the proportions of SA_PIPELINE_SPLIT (e.g.
    "9,9,2": a short last chunk keeps the exposed recurrence short at the
    end of the forward and the start of the backward).  Same math as
    unroll_core (the recurrence is sequential either way).
    """
    from .. import ops
    T, B = done.shape
    dev = frames.device
    main = torch.cuda.current_stream(dev)
    side = self._core_stream(dev)
    bounds = _chunk_bounds(T, chunks, measure_env('SA_PIPELINE_SPLIT'))
    fused = self.fused_core_ready(instr)
    F_in = self.core_input_size
    outs = []
    for k in range(len(bounds) - 1):
      t0, t1 = bounds[k], bounds[k + 1]
      n0, n1 = t0 * B, t1 * B
      ins = None
      if instr is not None:
        ins = (instr[0][n0:n1], instr[1][n0:n1])
      if fused:
        feats = self.conv_features(frames[n0:n1])
        instr_enc = (None if ins is None else
                     self.instruction_encoding(ins, n1 - n0, dev))
      else:
        x = self.core_inputs(frames[n0:n1], reward[n0:n1], actions[n0:n1],
                             ins).view(t1 - t0, B, -1)
      side.wait_stream(main)
      with torch.cuda.stream(side):
        if fused:
          # both side-stream inputs were produced on the main stream: their
          # blocks must not go back to the main stream's pool before the
          # side stream has read them
          feats.record_stream(side)
          if instr_enc is not None:
            instr_enc.record_stream(side)
          hs, state = ops.core_lstm(
              feats, self.linear_w, self.linear_b, self.lstm_kernel,
              self.lstm_bias, reward[n0:n1], actions[n0:n1], done[t0:t1],
              state, self.num_actions, instr_enc=instr_enc,
              # the gang recurrence beside the next chunk's torso: measured
              # experiment only (profiles/experiments.md round 6)
              allow_gang=measure_env('SA_PIPELINE_GANG') == '1')
        else:
          x.record_stream(side)
          hs, state = ops.lstm_unroll(
              x, done[t0:t1], state, self.lstm_kernel, self.lstm_bias,
              w_x=self.lstm_kernel[:F_in], w_h=self.lstm_kernel[F_in:],
              exact=self.compute_dtype == torch.float32)
      outs.append(hs)
    main.wait_stream(side)
    for h in outs:
      h.record_stream(main)
    for t in state:
      t.record_stream(main)
    return torch.cat(outs, 0), state

  def heads(self, core_out, task_ids=None):
    """task_ids: optional [B] task index per batch column (multi-head value
    with PopArt); without it a multi-head agent reports head 0."""
    logits = core_out @ self.policy_w + self.policy_b
    values = core_out @ self.baseline_w + self.baseline_b
    if self.num_value_heads == 1:
      return logits, values.squeeze(-1)
    if task_ids is None:
      return logits, values[..., 0]
    idx = task_ids.long().view(1, -1, 1).expand(values.shape[0], -1, 1)
    return logits, values.gather(-1, idx).squeeze(-1)

  # ------------------------------------------------------------------ API
  _inference_cache = None

  def inference_cache(self):
    """For an inference-only agent (InferenceModel): keep the fused core's
    per-step weight forms - W_h packed for the per-step LSTM kernel and, on
    the bf16 path, bf16 copies of the FC and W_x weights - refreshed by
    refresh_inference_cache() after every weight publish, so an inference
    step (and the board's captured graph) reads them instead of packing /
    casting them on every step.  No-op unless the fused core applies."""
    if not (self.fused_core_ready() and self.linear_w.is_cuda):
      return
    dev = self.lstm_kernel.device
    cache = {'w4': torch.empty(CORE_SIZE * 4 * CORE_SIZE, device=dev),
             'w16': None, 'w0pad': None}
    if (self.compute_dtype == torch.float32 and self.torso_kind == 'deep' and
        self.frame_shape[2] < 4):
      # the fp32 torso's stage-0 weights padded to the 4-channel image
      from ..ops.conv import deep_param_list
      w0 = deep_param_list(self)[0]
      cache['w0pad'] = torch.zeros(w0.shape[:2] + (4,) + w0.shape[3:],
                                   dtype=w0.dtype, device=dev)
    if self.compute_dtype == torch.bfloat16:
      bf = torch.bfloat16
      k_max = (self.core_input_size + 15) // 16 * 16
      cache['w16'] = (
          torch.empty(self.linear_w.shape, dtype=bf, device=dev),
          torch.empty(k_max, self.lstm_kernel.shape[1], dtype=bf, device=dev))
    self._inference_cache = cache
    self.refresh_inference_cache()

  @torch.no_grad()
  def refresh_inference_cache(self):
    """Re-packs / re-casts the cached weights (on the current stream)."""
    cache = self._inference_cache
    if cache is None:
      return
    from .. import ops
    ops.ext().lstm_pack_fwd(self.lstm_kernel[self.core_input_size:], cache['w4'])
    if cache['w0pad'] is not None:
      w0 = ops.conv.deep_param_list(self)[0]
      cache['w0pad'][:, :, :w0.shape[2]].copy_(w0)  # pad channels stay 0
    if cache['w16'] is not None:
      w16_fc, wx16 = cache['w16']
      w16_fc.copy_(self.linear_w)
      wx16.copy_(self.lstm_kernel[:wx16.shape[0]])

  def fused_core_ready(self, instr=None):
    """True when the HIP learner path (fused torso-FC/core-input/LSTM op,
    fused heads+V-trace loss) applies: HIP backend and a HIP torso (bf16
    kernels -> the bf16-operand core, exact-fp32 kernels -> the exact-fp32
    core of ops/core.py); the instruction encoding (language LSTM) joins the
    fused core input."""
    del instr
    return self.backend == 'hip' and _hip_torso_ready(self)

  def unroll_core(self, actions, env_outputs, core_state):
    """Everything of `unroll` up to the LSTM output: -> (core_out [T,B,256],
    core_state)."""
    reward, _, done, (frame, instr) = env_outputs
    T, B = actions.shape[0], actions.shape[1]
    frames = frame.reshape((T * B,) + tuple(frame.shape[2:]))
    if instr is not None:
      instr = (instr[0].reshape(T * B, -1), instr[1].reshape(T * B))
    done = done.to(torch.bool).view(T, B)
    chunks = min(self.pipeline_chunks, T // 4)
    if self.backend == 'hip' and frames.is_cuda and chunks > 1:
      return self._pipelined_core(
          frames, reward.reshape(T * B), actions.reshape(T * B), instr, done,
          core_state, chunks)
    if self.fused_core_ready(instr) and frames.is_cuda:
      from .. import ops
      feats = self.conv_features(frames)
      instr_enc = (None if instr is None else
                   self.instruction_encoding(instr, T * B, frames.device))
      cache = (self._inference_cache if not torch.is_grad_enabled() else None)
      return ops.core_lstm(feats, self.linear_w, self.linear_b,
                           self.lstm_kernel, self.lstm_bias,
                           reward.reshape(T * B), actions.reshape(T * B), done,
                           core_state, self.num_actions, instr_enc=instr_enc,
                           cache=cache)
    x = self.core_inputs(frames, reward.reshape(T * B),
                         actions.reshape(T * B), instr)
    x = x.view(T, B, -1)
    return self.core_unroll(x, done, core_state)

  def _fused_sampler_ready(self, core_out, task_ids, generator):
    """Heads + Gumbel-max sampling as one HIP kernel (actor_io.hip) when the
    caller drives a device-side PhiloxStream."""
    from ..ops.heads import PhiloxStream
    return (isinstance(generator, PhiloxStream) and self.backend == 'hip' and
            core_out.is_cuda and self.num_value_heads == 1 and
            task_ids is None and self.num_actions <= 32)

  def unroll(self, actions, env_outputs, core_state, sample=True,
             generator=None, task_ids=None):
    """Unrolls over T steps (experiment.py:219-237).

    actions: [T,B] last actions; env_outputs: StepOutput with [T,B,...]
    fields whose observation is (frame uint8 [T,B,H,W,C], instr or None).
    """
    T, B = actions.shape[0], actions.shape[1]
    core_out, core_state = self.unroll_core(actions, env_outputs, core_state)
    if sample and self._fused_sampler_ready(core_out, task_ids, generator):
      from .. import ops
      action, logits, baseline = ops.actor_heads_sample(
          core_out.reshape(T * B, -1), self.policy_w, self.policy_b,
          self.baseline_w, self.baseline_b, generator)
      return AgentOutput(action.view(T, B), logits.view(T, B, -1),
                         baseline.view(T, B)), core_state
    logits, baseline = self.heads(core_out, task_ids)
    if sample:
      probs = torch.softmax(logits.reshape(T * B, -1).float(), -1)
      action = torch.multinomial(probs, 1, generator=generator).view(T, B)
    else:
      action = None
    return AgentOutput(action, logits, baseline), core_state

  def step(self, last_action, env_output, core_state, generator=None):
    """Single batched step for actors: inputs [B,...] -> outputs [B,...]."""
    exp = lambda t: None if t is None else t.unsqueeze(0)
    reward, info, done, (frame, instr) = env_output
    if instr is not None:
      instr = (instr[0].unsqueeze(0), instr[1].unsqueeze(0))
    eo = (exp(reward), info, exp(done), (exp(frame), instr))
    out, state = self.unroll(exp(last_action), eo, core_state,
                             generator=generator)
    return AgentOutput(out.action[0], out.policy_logits[0],
                       out.baseline[0]), state
