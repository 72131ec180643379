"""`VFDepthAlgo` — drop-in for `/root/reference/models/vfdepth.py:20-320` on MI355X.

Same constructor `VFDepthAlgo(cfg, rank)`, same `process_batch(inputs, rank) -> (outputs, losses)`
contract and schemas, same optimizer / scheduler / DDP(+SyncBN) wiring,
dataloader accessors, train/val switches and checkpoint I/O.  The step itself is restructured
for the GPU:

* all six cameras are rendered (K4) and scored (K5) in one launch sequence instead of a Python
  loop over cameras x warps (the per-camera module APIs remain available);
* no host synchronisation inside the step: loss logs are device tensors, the reference's
  data-dependent branches (empty-overlap skip, non-finite clamp) are resolved on the device;
* the identity-loss tie-break noise comes from an in-kernel counter RNG (`noise_mode='device'`,
  default) or, for bit-level parity with the reference, from the CPU global RNG exactly as the
  reference draws it (`noise_mode='cpu_global'`).
"""
import contextlib
import gc
import os
import sys
from collections import defaultdict

import torch
import torch.distributed as dist
import torch.nn.functional as F
import torch.optim as optim
from torch.utils._python_dispatch import TorchDispatchMode
from torch.utils.data import DataLoader

from . import fusion
from .config import flatten
from .geometry import Pose, ViewRendering, inverse4x4
from .losses import DepthSynLoss, MultiCamLoss, SingleCamLoss
from .network import FusedDepthNet, FusedPoseNet, MonoDepthNet, MonoPoseNet
from .rotation import _qm_consts
from .synth import SyntheticSurroundDataset

_NO_DEVICE_KEYS = ['idx', 'dataset_idx', 'sensor_name', 'filename']
_OPTIMIZER_NAME = 'adam'


def _record_stream(obj, stream):
    """record_stream(stream) on every CUDA tensor of a nested dict / list / tuple."""
    if torch.is_tensor(obj):
        if obj.is_cuda:
            obj.record_stream(stream)
    elif isinstance(obj, dict):
        for v in obj.values():
            _record_stream(v, stream)
    elif isinstance(obj, (list, tuple)):
        for v in obj:
            _record_stream(v, stream)


def _trace(what, sync=True):
    """VFD_GRAPH_TRACE=1: a line per stage of graphed_train_step (after a device sync when allowed),
    so a crash is attributed to its stage."""
    if os.environ.get('VFD_GRAPH_TRACE') == '1':
        if sync:
            torch.cuda.synchronize()
        print(f'[graph] {what}', file=sys.stderr, flush=True)


def _detach_all(obj):
    """The same nested dict / list / tuple with every tensor detached (views of the same memory)."""
    if torch.is_tensor(obj):
        return obj.detach()
    if isinstance(obj, dict):
        return {k: _detach_all(v) for k, v in obj.items()}
    if isinstance(obj, (list, tuple)):
        return type(obj)(_detach_all(v) for v in obj)
    return obj


class _CaptureCheck(TorchDispatchMode):
    """VFD_GRAPH_CHECK=1: every framework op of the captured step whose tensors are on both the host
    and the device is recorded.  A host->device copy inside a capture is a graph node that reads the
    host buffer at every replay — long after the temporary it copied from was freed — and its value
    is frozen at the capture step's.  The captured step must have none."""

    def __init__(self):
        super().__init__()
        self.found = []

    def __torch_dispatch__(self, func, types, args=(), kwargs=None):
        out = func(*args, **(kwargs or {}))
        devs = set()
        for t in torch.utils._pytree.tree_leaves((args, kwargs or {}, out)):
            if torch.is_tensor(t):
                devs.add(t.device.type)
        if 'cpu' in devs and 'cuda' in devs:
            shapes = [tuple(t.shape) for t in torch.utils._pytree.tree_leaves(args) if torch.is_tensor(t)]
            self.found.append(f'{func} {shapes}')
        return out

    def live_graph_before_capture(self):
        """Tensors of an earlier step's autograd graph still alive when the capture starts keep
        that step's AccumulateGrad nodes (and their stream) in use by the captured backward."""
        import gc
        gc.collect()
        for o in gc.get_objects():
            try:
                if torch.is_tensor(o) and o.grad_fn is not None:
                    self.found.append(f'live autograd graph before capture: {tuple(o.shape)} {type(o.grad_fn).__name__}')
            except Exception:       # objects that refuse inspection
                continue

    def raise_if_any(self):
        if self.found:
            raise RuntimeError('host<->device transfers inside the captured step:\n  ' + '\n  '.join(self.found[:20]))


class VFDepthAlgo:
    def __init__(self, cfg, rank):
        self.cfg = cfg
        self.rank = rank
        self._dataloaders = {}
        self.mode = None
        self.ddp_enable = False
        for k, v in flatten(cfg).items():
            setattr(self, k, v)
        self.device = torch.device(f'cuda:{rank}') if isinstance(rank, int) else torch.device(rank)
        if self.device.type == 'cuda':
            # the C-ABI ops launch on the current device's stream: make it this rank's device
            torch.cuda.set_device(self.device)
        if torch.backends.cudnn.deterministic:
            # the reference's train.py:23 switch; MIOpen honours it only through this variable,
            # read once per process at its first convolution (so set it before building models)
            os.environ.setdefault('MIOPEN_DEBUG_CONVOLUTION_DETERMINISTIC', '1')
        if getattr(self, 'net_precision', 'fp32') not in ('fp32', 'bf16'):
            raise ValueError(f'net_precision must be fp32 or bf16, got {self.net_precision!r}')
        self.prepare_dataset(cfg, rank)
        self.models = self.prepare_model(cfg, rank)
        self.losses = self.init_losses(cfg, rank)
        self.view_rendering, self.pose = ViewRendering(cfg, rank), Pose(cfg)
        self.set_optimizer()
        if self.pretrain and rank == 0:
            self.load_weights()

    # ------------------------------------------------------------------ construction
    def init_losses(self, cfg, rank):
        if self.aug_depth:
            return DepthSynLoss(cfg, rank)
        if self.spatio_temporal or self.spatio:
            return MultiCamLoss(cfg, rank)
        return SingleCamLoss(cfg, rank)

    def prepare_model(self, cfg, rank):
        models = {
            'pose_net': (FusedPoseNet(cfg) if self.pose_model == 'fusion' else MonoPoseNet(cfg)).to(self.device),
            'depth_net': (FusedDepthNet(cfg) if self.depth_model == 'fusion' else MonoDepthNet(cfg)).to(self.device),
        }
        if self.ddp_enable:
            from torch.nn.parallel import DistributedDataParallel as DDP
            on_gpu = self.device.type == 'cuda'
            for k, v in models.items():
                # one SyncBatchNorm group per net (created in the same order on every rank): the
                # pose branch runs on its own stream, and its BN collectives then go to their own
                # communicator (and stream) instead of queueing behind the depth branch's
                group = dist.new_group(list(range(self.world_size)))
                # torch's SyncBatchNorm only runs on GPU modules: the gloo/CPU rehearsal keeps
                # per-rank BatchNorm, the GPU path converts exactly as the reference does
                if on_gpu:
                    v = torch.nn.SyncBatchNorm.convert_sync_batchnorm(v, group)
                # broadcast_buffers as the reference (vfdepth.py:70) — except at world size 1, where
                # the broadcast is a self-copy whose in-place version bump on the BatchNorm running
                # stats (saved by MIOpen's batch-norm backward) breaks the second pose-net call of
                # the step; at world > 1 SyncBatchNorm's synchronised path saves no running stats
                # ddp.graph_capture: built with the capture stream current, so the AccumulateGrad
                # nodes (and DDP's hooks) live on a stream a HIP graph can capture (_capture_stream)
                cap = on_gpu and bool(cfg['ddp'].get('graph_capture', False))
                with (torch.cuda.stream(self._capture_stream()) if cap else contextlib.nullcontext()):
                    models[k] = DDP(v, device_ids=[self.device.index] if on_gpu else None,
                                    broadcast_buffers=self.world_size > 1)
                self._ddp_on_capture_stream = cap
        return models

    def _dataset(self, cfg, mode, with_depth):
        """The on-disk DDAD / NuScenes reader (`data.construct_dataset`, base_dataset.py:5-50) when
        `data.data_path` names a dataset, else the synthetic DDAD-shaped generator."""
        if str(cfg['data'].get('data_path', 'synthetic')) != 'synthetic':
            from .data import augmentation, construct_dataset
            return construct_dataset(cfg, 'train' if mode == 'train' else 'val', **augmentation(cfg, mode))
        if mode == 'val':
            return SyntheticSurroundDataset(cfg, length=8, seed=7, with_depth=True)
        return SyntheticSurroundDataset(cfg, with_depth=with_depth)

    def prepare_dataset(self, cfg, rank):
        if self.mode == 'eval' or cfg['model'].get('mode') == 'eval':
            self._dataloaders['eval'] = DataLoader(self._dataset(cfg, 'eval', True),
                                                   batch_size=self.eval_batch_size, shuffle=False, drop_last=True)
            return
        ds = self._dataset(cfg, 'train', False)
        opts = {'batch_size': self.batch_size, 'shuffle': not self.ddp_enable, 'num_workers': self.num_workers,
                'pin_memory': True, 'drop_last': True}
        if self.ddp_enable:
            # rank may be a device (CPU rehearsal): the sampler wants the process rank
            prank = rank if isinstance(rank, int) else (dist.get_rank() if dist.is_initialized() else 0)
            self.train_sampler = torch.utils.data.distributed.DistributedSampler(
                ds, num_replicas=self.world_size, rank=prank, shuffle=True)
            opts['sampler'] = self.train_sampler
        self._dataloaders['train'] = DataLoader(ds, **opts)
        if rank == 0:
            self._dataloaders['val'] = DataLoader(self._dataset(cfg, 'val', True),
                                                  batch_size=self.batch_size, shuffle=False, drop_last=True)
        self.num_total_steps = len(ds) // (self.batch_size * self.world_size) * self.num_epochs

    def set_optimizer(self, capturable=False):
        params = []
        for m in self.models.values():
            params += list(m.parameters())
        fused = self.device.type == 'cuda'
        capturable = capturable and fused
        # a captured step reads the learning rate from device memory: a tensor lr, which
        # StepLR updates in place (fill_), so the scheduler's decay reaches graph replays
        lr = torch.tensor(float(self.learning_rate), device=self.device) if capturable else self.learning_rate
        self.optimizer = optim.Adam(params, lr, fused=fused, capturable=capturable)
        self.lr_scheduler = optim.lr_scheduler.StepLR(self.optimizer, self.scheduler_step_size, 0.1)

    # ------------------------------------------------------------------ base-model API
    def train_dataloader(self):
        return self._dataloaders['train']

    def val_dataloader(self):
        return self._dataloaders['val']

    def eval_dataloader(self):
        return self._dataloaders['eval']

    def set_train(self):
        self.mode = 'train'
        for m in self.models.values():
            m.train()

    def set_val(self):
        self.mode = 'val'
        for m in self.models.values():
            m.eval()

    def save_model(self, epoch):
        path = os.path.join(self.save_weights_root, f'weights_{epoch}')
        os.makedirs(path, exist_ok=True)
        for name, m in self.models.items():
            torch.save(m.state_dict(), os.path.join(path, f'{name}.pth'))
        torch.save(self.optimizer.state_dict(), os.path.join(path, f'{_OPTIMIZER_NAME}.pth'))

    def load_weights(self):
        """base_model.py:58-93: filtered state-dict load per model; the Adam state only in train
        mode, and a param-group mismatch (ValueError) keeps a fresh optimizer, as the reference."""
        assert os.path.isdir(self.load_weights_dir), f'\tCannot find {self.load_weights_dir}'
        print(f'Loading a model from {self.load_weights_dir}')
        for name in self.models_to_load:
            path = os.path.join(self.load_weights_dir, f'{name}.pth')
            model = self.models[name]
            own = model.state_dict()
            src = torch.load(path, map_location=self.device, weights_only=True)
            own.update({k: v for k, v in src.items() if k in own})
            model.load_state_dict(own)
        if self.mode != 'train':
            return
        opt = os.path.join(self.load_weights_dir, f'{_OPTIMIZER_NAME}.pth')
        if not os.path.isfile(opt):
            print(f'\tCannot find {_OPTIMIZER_NAME} weights, so the optimizer will be randomly initialized')
            return
        try:
            self.optimizer.load_state_dict(torch.load(opt, map_location=self.device, weights_only=True))
        except ValueError:
            print(f'\tCannnot load {_OPTIMIZER_NAME} - the optimizer will be randomly initialized')

    # ------------------------------------------------------------------ step
    def process_batch(self, inputs, rank, noise=None):
        """Move the batch to the device, estimate poses/depths, render and score every camera.

        `noise` (optional, [N, B, T, H, W]) overrides the identity-loss noise (parity tests)."""
        fusion.begin_step()
        for key, ipt in list(inputs.items()):
            if key in _NO_DEVICE_KEYS or not torch.is_tensor(ipt) and not isinstance(ipt, list):
                continue
            if isinstance(key, str) and 'context' in key:
                inputs[key] = [t.float().to(self.device, non_blocking=True) for t in ipt]
            elif torch.is_tensor(ipt):
                inputs[key] = ipt.float().to(self.device, non_blocking=True)
        outputs = self.estimate_vfdepth(inputs)
        losses = self.compute_losses(inputs, outputs, noise)
        return outputs, losses

    def _branch_stream(self):
        """Second stream for the pose branch of a training step (default; VFD_BRANCH_STREAMS=0 turns
        it off): the pose net (its encoder over the frame pairs, K2 / K2C, decoder) and the depth net
        are independent until the view synthesis, so their many small latency-bound kernels
        (small-layer BN, small convs) fill each other's idle CUs — config 2 27.55 vs 30.27-30.50
        ms/step on one box (round 5).  Under DDP the collectives of both branches (SyncBN, DDP's
        buckets) go to the process group's own stream in host issue order, which is the same on every
        rank.  Grad mode only.  Under HIP-graph capture the branch stream is forked from the capture
        stream and joined back (forward: `estimate_vfdepth`; backward: autograd's leaf-stream sync and
        `_join_branch`), so the captured step has the same two-branch schedule as the eager one."""
        if (self.device.type != 'cuda' or os.environ.get('VFD_BRANCH_STREAMS', '1') == '0'
                or not getattr(self, 'branch_streams', True) or not torch.is_grad_enabled()
                or self.pose_model != 'fusion' or self.depth_model != 'fusion'):
            return None
        if torch.cuda.is_current_stream_capturing() and dist.is_initialized() and dist.get_world_size() > 1:
            # a capture at world > 1: the pose branch's SyncBatchNorm all-reduces would make the
            # branch stream and the process group's stream wait on each other, which this HIP
            # runtime turns into a parent/child cycle of capture streams (kernels._wait_stream)
            return None
        if getattr(self, '_bstream', None) is None:
            self._bstream = torch.cuda.Stream(self.device)
        return self._bstream

    def _join_branch(self):
        """Make the current stream wait for the pose branch's stream if THIS step used it (its
        backward ran there).  Only then: under capture, waiting on a stream the capture never forked
        would be a cross-capture dependency (hipErrorStreamCaptureIsolation)."""
        if getattr(self, '_branch_live', False):
            torch.cuda.current_stream(self.device).wait_stream(self._bstream)
            self._branch_live = False

    def estimate_vfdepth(self, inputs):
        inputs['extrinsics_inv'] = inverse4x4(inputs['extrinsics'])
        outputs = {('cam', c): {} for c in range(self.num_cams)}
        side = self._branch_stream()
        if side is not None:
            # the geometry both fusion nets share (1/8 mask, K2 plan object) made on this stream first
            dn = self.models['depth_net']
            vf = getattr(dn, 'module', dn).fusion_net
            vf._plan(inputs, vf.space(self.device))
            main = torch.cuda.current_stream(self.device)
            side.wait_stream(main)
            self._branch_live = True
            with torch.cuda.stream(side):
                pose_pred = self.predict_pose(inputs)
            depth_feats = self.predict_depth(inputs)
            main.wait_stream(side)
            _record_stream(pose_pred, main)     # side-stream tensors read on this stream from here on
        else:
            pose_pred = self.predict_pose(inputs)
            depth_feats = self.predict_depth(inputs)
        packed = depth_feats.pop('_packed', None)
        packed_aug = depth_feats.pop('_packed_aug', None)
        if '_extrinsics_aug' in depth_feats:          # written by VFNet (travels through DDP)
            inputs['extrinsics_aug'] = depth_feats.pop('_extrinsics_aug')
        if '_cam_T_cam' in pose_pred:                 # batched poses of the fusion pose model
            outputs['_cam_T_cam'] = pose_pred['_cam_T_cam']
        for c in range(self.num_cams):
            outputs[('cam', c)].update(pose_pred[('cam', c)])
            outputs[('cam', c)].update(depth_feats[('cam', c)])
        self.compute_depth_maps(inputs, outputs, packed, packed_aug)
        return outputs

    def _net(self, name):
        net = self.models[name]
        if self.mode != 'train' and self.ddp_enable:
            net = net.module
        return net

    def predict_pose(self, inputs):
        return self.pose.compute_pose(self._net('pose_net'), inputs)

    def predict_depth(self, inputs):
        net = self._net('depth_net')
        if self.depth_model == 'fusion':
            return net(inputs)
        return {('cam', c): net(inputs[('color_aug', 0, 0)][:, c]) for c in range(self.num_cams)}

    def to_depth(self, disp_in, K_in):
        """disp -> metric-scaled depth (vfdepth.py:277-288)."""
        lo, hi = 1 / self.max_depth, 1 / self.min_depth
        if tuple(disp_in.shape[-2:]) != (self.height, self.width):
            disp_in = F.interpolate(disp_in, [self.height, self.width], mode='bilinear', align_corners=False)
        depth = 1 / (lo + (hi - lo) * disp_in)
        return depth * K_in[:, 0:1, 0:1].unsqueeze(2) / self.focal_length_scale      # (depth * fx) / fls

    def compute_depth_maps(self, inputs, outputs, packed=None, packed_aug=None):
        """Per-camera depth (vfdepth.py:263-275), and the augmented view's (aug_depth); with the
        packed [B*N] decoder output the depth of all cameras is one elementwise op, kept as
        [B, N, H, W] for the kernels."""
        K0 = inputs[('K', 0)]
        B, N = K0.shape[:2]
        variants = [('', packed)] + ([('aug', packed_aug)] if self.aug_depth else [])
        for tag, pk in variants:
            sfx = (tag,) if tag else ()
            disp_all = outputs.setdefault('_disp_aug_all' if tag else '_disp_all', {})
            depth_all = outputs.setdefault('_depth_aug_all' if tag else '_depth_all', {})
            for scale in self.scales:
                key = ('disp', scale)
                if pk is not None and key in pk:
                    disp = pk[key].view(B, N, *pk[key].shape[1:])[:, :, 0]
                else:
                    disp = torch.stack([outputs[('cam', c)][key + sfx][:, 0] for c in range(N)], 1)
                if tuple(disp.shape[-2:]) != (self.height, self.width):
                    disp_f = F.interpolate(disp, [self.height, self.width], mode='bilinear', align_corners=False)
                else:
                    disp_f = disp
                lo, hi = 1 / self.max_depth, 1 / self.min_depth
                depth = 1 / (lo + (hi - lo) * disp_f)
                depth = depth * K0[:, :, 0:1, 0:1] / self.focal_length_scale
                disp_all[scale] = disp
                depth_all[scale] = depth
                for c in range(N):
                    outputs[('cam', c)][('depth', scale) + sfx] = depth[:, c].unsqueeze(1)

    def compute_losses(self, inputs, outputs, noise=None):
        # with the batched fusion poses every warp matrix comes from one batched chain (rel None)
        rel = (None if '_cam_T_cam' in outputs else
               {c: self.pose.compute_relative_cam_poses(inputs, outputs, c) for c in range(self.num_cams)})
        packed = self.view_rendering.render_all(inputs, outputs, rel, outputs['_depth_all'])
        if self.aug_depth:
            outputs['_tform'] = self.view_rendering.render_depth_synthesis(
                inputs, outputs, outputs['_depth_all'][0], outputs['_depth_aug_all'][0])
        total, logs = self.losses.forward_all(inputs, outputs, packed, outputs['_disp_all'], outputs['_depth_all'], noise)
        losses = dict(logs)
        losses['total_loss'] = total
        return losses

    # ------------------------------------------------------------------ HIP graph
    def train_step(self, inputs):
        """zero_grad -> process_batch -> backward -> optimizer step (vfdepth_trainer.py:63-66).
        Returns the losses DETACHED: a caller that keeps them (a logger, the bench) must not keep the
        step's autograd graph alive — its AccumulateGrad nodes, and the streams they were created
        on, would otherwise carry into later steps (and into a graph capture)."""
        self.optimizer.zero_grad(set_to_none=True)
        _, losses = self.process_batch(inputs, self.rank)
        losses['total_loss'].backward()
        self._join_branch()
        self.optimizer.step()
        return {k: (v.detach() if torch.is_tensor(v) else v) for k, v in losses.items()}

    def _capture_stream(self):
        """The stream a captured step warms up and is captured on (created once).  Under DDP with
        `ddp.graph_capture` the DDP wrappers are BUILT with it current (prepare_model): DDP's reducer
        creates and keeps every parameter's AccumulateGrad node at construction, and autograd
        accumulates each gradient (and fires DDP's all-reduce hooks) on the stream its node was
        created on — on the legacy default stream, which cannot join a capture (round 6:
        hipErrorStreamCaptureImplicit in the captured backward), unless DDP was built on this one."""
        if getattr(self, '_cap_stream', None) is None:
            self._cap_stream = torch.cuda.Stream(self.device)
        return self._cap_stream

    def graphed_train_step(self, batch, warmup=3):
        """Capture one whole training step (forward, losses, backward, Adam) in a HIP graph.

        Returns step(new_batch=None) -> losses (detached): copies new_batch (same shapes) into the
        static input buffers and replays the graph: ~1100 kernel launches per step become one.
        Needs a capturable optimizer (set_optimizer(capturable=True)).  The captured step is the
        eager default one: batched frame pairs and the pose branch on its own stream (forked from
        and joined back into the capture stream).  The warm-up steps run in that same configuration
        on the capture stream itself, so every MIOpen problem is found / compiled before the capture
        and every AccumulateGrad node lives on a captured stream.

        Under DDP (trainer/vfdepth_trainer.py:61-66 with models/vfdepth.py:56-71's wrapping) the
        config must set `ddp.graph_capture: True` (the wrappers are then built on the capture
        stream, `_capture_stream`), and the captured step holds DDP's
        bucketed gradient all-reduces and the fused BN's SyncBatchNorm all-reduces (RCCL kernels on
        the ranks' streams, captured with the step): DDP settles its buckets during its first
        iterations, so at least 11 eager DDP steps run before the capture, as PyTorch requires.
        Every rank captures and replays the same step, so the collectives stay matched."""
        if self.ddp_enable:
            warmup = max(warmup, 11)
        static = {k: (v.to(self.device) if torch.is_tensor(v) else v) for k, v in batch.items()}
        self.losses.device_seed = True
        # no autograd graph of an earlier step may survive into the warm-up or the capture: its
        # AccumulateGrad nodes would carry their stream into the captured backward
        gc.collect()
        if self.ddp_enable and not getattr(self, '_ddp_on_capture_stream', False):
            raise RuntimeError('graphed_train_step under DDP needs the DDP wrappers built on the capture '
                               'stream: set cfg["ddp"]["graph_capture"] = True before constructing VFDepthAlgo')
        if self.ddp_enable and (os.environ.get('TORCH_NCCL_CUDA_EVENT_CACHE') != '0'
                                or os.environ.get('TORCH_NCCL_ASYNC_ERROR_HANDLING') != '0'):
            # the process group's watchdog polls its works' events; pooled events re-recorded inside
            # the capture make that poll fail (hipErrorCapturedEvent aborts the process, round 6)
            raise RuntimeError('graphed_train_step under DDP: export TORCH_NCCL_CUDA_EVENT_CACHE=0 and '
                               'TORCH_NCCL_ASYNC_ERROR_HANDLING=0 before init_process_group')
        cap = self._capture_stream()                  # warm-up AND capture stream
        cap.wait_stream(torch.cuda.current_stream(self.device))
        with torch.cuda.stream(cap):
            for i in range(warmup):
                self.train_step(dict(static))
                _trace(f'warm-up step {i}')
        torch.cuda.current_stream(self.device).wait_stream(cap)
        # constants the captured step builds on the device (the augmented view's rotation is drawn
        # on the device generator under capture): made here, so no host->device copy is captured
        _qm_consts(self.device, torch.float32)
        gc.collect()
        graph = torch.cuda.CUDAGraph()
        dump = os.environ.get('VFD_GRAPH_DUMP')          # diagnostics: the captured graph as DOT
        if dump:
            graph.enable_debug_mode()
        self.optimizer.zero_grad(set_to_none=True)
        check = _CaptureCheck() if os.environ.get('VFD_GRAPH_CHECK') == '1' else contextlib.nullcontext()
        if isinstance(check, _CaptureCheck):
            check.live_graph_before_capture()
        _trace(f'capture begins on stream {cap.cuda_stream:#x}, branch stream '
               f'{getattr(getattr(self, "_bstream", None), "cuda_stream", 0):#x}, default stream '
               f'{torch.cuda.default_stream(self.device).cuda_stream:#x}')
        # under a process group, its watchdog thread polls the events of finished collectives while
        # the capture runs; in the default 'global' mode any thread's event query during a capture
        # fails (hipErrorStreamCaptureUnsupported, and the watchdog aborts the process: round 6,
        # intermittent), so the capture checks only this thread's calls ('thread_local').  The step
        # itself is capture-clean in 'global' mode (every single-process capture runs that way).
        mode = 'thread_local' if dist.is_available() and dist.is_initialized() else 'global'
        with torch.cuda.graph(graph, stream=cap, capture_error_mode=mode):
            with check:
                try:
                    static_outputs, static_losses = self.process_batch(dict(static), self.rank)
                    _trace('captured forward', sync=False)
                    static_losses['total_loss'].backward()
                    _trace('captured backward', sync=False)
                    self._join_branch()
                    self.optimizer.step()
                    _trace('captured optimizer step', sync=False)
                except BaseException:
                    # the runtime may not survive ending an invalidated capture: report first
                    import traceback
                    traceback.print_exc()
                    sys.stderr.flush()
                    raise
        _trace('capture ended')
        if isinstance(check, _CaptureCheck):
            check.raise_if_any()
        if dump:
            graph.debug_dump(dump)
        # keep only detached views: the captured step's autograd graph (and its AccumulateGrad nodes)
        # must not outlive the capture
        static_losses = {k: (v.detach() if torch.is_tensor(v) else v) for k, v in static_losses.items()}
        static_outputs = _detach_all(static_outputs)

        def step(new_batch=None):
            if new_batch is not None:
                for k, v in new_batch.items():
                    if torch.is_tensor(v) and torch.is_tensor(static.get(k)):
                        static[k].copy_(v, non_blocking=True)
            graph.replay()
            return static_losses

        step.graph = graph
        step.outputs = static_outputs      # refreshed by every replay
        return step

    def compute_depth_metrics(self, inputs, outputs, vis_scale=False):
        """Abs.Rel & co. against inputs['depth'] (Logger.compute_depth_losses, logger.py:193-247)."""
        from .metrics import compute_depth_losses
        ev = self.cfg.get('eval', {})
        lo, hi = float(ev.get('eval_min_depth', 0.0)), float(ev.get('eval_max_depth', 200.0))
        metric, median, scales = compute_depth_losses(inputs, outputs, self.num_cams, lo, hi, return_scales=True)
        if vis_scale:
            print(f'          | median scale = {scales}')
        return metric, median

    def pred_cam_imgs(self, inputs, outputs, cam):
        """Reference per-camera API (vfdepth.py:315-320)."""
        self.view_rendering(inputs, outputs, cam, self.pose.compute_relative_cam_poses(inputs, outputs, cam))

    def compute_losses_per_camera(self, inputs, outputs, noise=None):
        """The reference's camera loop (vfdepth.py:290-313) on the per-camera kernel entry points."""
        total = 0
        fn = defaultdict(list)
        for c in range(self.num_cams):
            self.pred_cam_imgs(inputs, outputs, c)
            cl, ld = self.losses(inputs, outputs, c, None if noise is None else noise[c:c + 1])
            total = total + cl
            for k, v in ld.items():
                fn[k].append(v)
        out = {k: sum(v) / float(len(v)) for k, v in fn.items()}
        out['total_loss'] = total / self.num_cams
        return out
