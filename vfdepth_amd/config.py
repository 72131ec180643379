"""Configuration schema of the VFDepth training step.

Mirrors the reference's nested-YAML config (`/root/reference/utils/misc.py:44-72`,
canonical values `/root/reference/configs/ddad/ddad_surround_fusion.yaml:1-97`):
every section is a plain dict, derived keys (`num_cams`, `rel_cam_list`, `mode`, log
paths) are added the same way so a reference config file drops in unchanged.
"""
import copy
import os

import yaml

# Camera naming tables (reference utils/misc.py:8-10).  Index = rig position:
#            3 1
#   rear <- 5   0 -> front
#            4 2
NUSC_CAMERAS = ['CAM_FRONT', 'CAM_FRONT_LEFT', 'CAM_FRONT_RIGHT',
                'CAM_BACK_LEFT', 'CAM_BACK_RIGHT', 'CAM_BACK']
DDAD_CAMERAS = ['camera_01', 'camera_05', 'camera_06', 'camera_07', 'camera_08', 'camera_09']
# spatial neighbours of every rig position (reference utils/misc.py:10)
NEIGHBOURS = {0: (1, 2), 1: (0, 3), 2: (0, 4), 3: (1, 5), 4: (2, 5), 5: (3, 4)}


def camera_indices(cameras):
    """Rig position of each camera name (reference utils/misc.py:13-26); None if unknown."""
    out = []
    for name in cameras:
        if name in DDAD_CAMERAS:
            out.append(DDAD_CAMERAS.index(name))
        elif name in NUSC_CAMERAS:
            out.append(NUSC_CAMERAS.index(name))
        else:
            out.append(None)
    return out


def relative_cameras(cameras):
    """Neighbour list per present camera (reference utils/misc.py:29-41)."""
    present = camera_indices(cameras)
    table = {}
    for idx in present:
        table[idx] = [n for n in NEIGHBOURS[idx] if n in present]
    return table


def _derive(cfg, cfg_name, mode, weight_path):
    data = cfg['data']
    log_path = os.path.join(data.get('log_dir', './results/'), cfg_name)
    data['log_path'] = log_path
    data['save_weights_root'] = os.path.join(log_path, 'models')
    if weight_path is None:
        weight_path = os.path.join(log_path, 'models', cfg.get('load', {}).get('weights', 'weights_0'))
    data['load_weights_dir'] = weight_path
    data['num_cams'] = len(data['cameras'])
    data['rel_cam_list'] = relative_cameras(data['cameras'])
    cfg['model']['mode'] = mode
    if mode == 'train':
        cfg.setdefault('eval', {})['syn_visualize'] = False
    elif mode == 'eval':
        cfg['ddp']['world_size'] = 1
        cfg['ddp']['gpus'] = [0]
        cfg['training']['batch_size'] = cfg['eval']['eval_batch_size']
        cfg['training']['depth_flip'] = False
    return cfg


def get_config(config, mode='train', weight_path=None):
    """Load a reference-format YAML file (or take a dict) and add the derived keys."""
    if isinstance(config, dict):
        cfg = copy.deepcopy(config)
        name = 'inline'
    else:
        with open(config, 'r') as fh:
            cfg = yaml.load(fh, Loader=yaml.SafeLoader)
        name = os.path.splitext(os.path.basename(config))[0]
    return _derive(cfg, name, mode, weight_path)


def surround_fusion_cfg(**over):
    """`ddad_surround_fusion.yaml` as a dict (values: reference configs/ddad/ddad_surround_fusion.yaml).

    Keyword overrides are `section__key=value` or plain `key=value` (searched in every section).
    """
    cfg = {
        'ddp': {'ddp_enable': False, 'world_size': 1, 'gpus': [0]},
        'model': {
            'num_layers': 18, 'weights_init': False,
            'depth_model': 'fusion', 'pose_model': 'fusion',
            'fusion_level': 2, 'fusion_feat_in_dim': 256, 'use_skips': False,
            'voxel_unit_size': [1.0, 1.0, 1.5], 'voxel_size': [100, 100, 20],
            'voxel_str_p': [-50.0, -50.0, -15.0], 'voxel_pre_dim': [64],
            'proj_d_bins': 50, 'proj_d_str': 2, 'proj_d_end': 50,
        },
        'data': {
            'data_path': 'synthetic', 'log_dir': './results/', 'dataset': 'ddad',
            'back_context': 1, 'forward_context': 1, 'depth_type': 'lidar',
            'cameras': list(DDAD_CAMERAS),
            'train_requirements': '(gt_pose, mask)', 'val_requirements': '(gt_pose, gt_depth, mask)',
        },
        'training': {
            'height': 384, 'width': 640, 'scales': [0], 'frame_ids': [0, -1, 1],
            'batch_size': 1, 'num_workers': 0, 'learning_rate': 0.0001,
            'num_epochs': 20, 'scheduler_step_size': 15,
            'min_depth': 1.5, 'max_depth': 200.0,
            'spatio': True, 'spatio_temporal': True, 'intensity_align': True,
            'focal_length_scale': 300, 'aug_depth': False, 'aug_angle': [15, 15, 40],
            # build-only: precision of the dense nets (encoders/decoders/reduce_dim on MIOpen);
            # 'bf16' = autocast for config 3, the HIP fusion/geometry/loss kernels stay fp32
            'net_precision': 'fp32',
        },
        'loss': {'disparity_smoothness': 0.001, 'spatio_coeff': 0.03,
                 'spatio_tempo_coeff': 0.1, 'pose_loss_coeff': 0.0},
        'eval': {'eval_batch_size': 4, 'eval_num_workers': 0, 'eval_min_depth': 0,
                 'eval_max_depth': 200, 'eval_visualize': False, 'syn_visualize': False,
                 'syn_idx': 0},
        'load': {'pretrain': False, 'weights': 'weights_19', 'models_to_load': ['depth_net']},
        'logging': {'early_phase': 2000, 'log_frequency': 100, 'late_log_frequency': 1000,
                    'save_frequency': 1},
    }
    apply_overrides(cfg, **over)
    return get_config(cfg)


def mono_cfg(**over):
    """Config 1 of BASELINE.json: fsm baseline nets, 1 camera, temporal loss only."""
    cfg = surround_fusion_cfg()
    cfg['model'].update({'depth_model': 'fsm', 'pose_model': 'fsm'})
    cfg['data']['cameras'] = [DDAD_CAMERAS[0]]
    cfg['training'].update({'height': 128, 'width': 192, 'spatio': False, 'spatio_temporal': False})
    cfg['loss'].update({'disparity_smoothness': 0.1, 'pose_loss_coeff': 0.1})
    apply_overrides(cfg, **over)
    return get_config(cfg)


def apply_overrides(cfg, **over):
    for key, val in over.items():
        if '__' in key:
            sec, k = key.split('__', 1)
            cfg[sec][k] = val
            continue
        for sec in cfg.values():
            if isinstance(sec, dict) and key in sec:
                sec[key] = val
                break
        else:
            raise KeyError(f'unknown config key {key!r}')
    return cfg


def flatten(cfg):
    """All sections merged into one namespace, as every reference class does in `read_config`."""
    flat = {}
    for sec in cfg.values():
        if isinstance(sec, dict):
            flat.update(sec)
    return flat
