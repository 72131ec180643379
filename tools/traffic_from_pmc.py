"""Per-op HBM traffic from rocprofv3 PMC passes (FETCH_SIZE and WRITE_SIZE in separate runs).

    python tools/traffic_from_pmc.py <fetch_counter_collection.csv> <write_counter_collection.csv> > profiles/traffic_config2.json

Per MI355X_MICROARCH.md (HBM / rocprofv3): FETCH_SIZE and WRITE_SIZE are in KiB; on gfx950
FETCH_SIZE reports 1/2 of the bytes of coalesced reads — calibrated here for 4-, 8- and 16-B
lanes alike on a known-byte probe (tools/probe_fetch.py: 0.5000 of 512 MiB for all three widths,
profiles/r2/fetch_probe.json) — so it is doubled; WRITE_SIZE is taken as is.  Each op (a C-ABI call, as the bench's roofline names it) sums the kernels it
launches; values are bytes per op launch, averaged over all launches in the run."""
import collections
import csv
import json
import re
import sys

OPS = {
    'mask_downsample': ['mask_downsample_k'],
    'fusion_plan': ['fusion_plan_k', 'plan_index_k', 'plan_count_k', 'plan_scan_k', 'plan_fill_k', 'plan_order_k',
                    'plan_copy_k', 'plan_task_k'],
    'fuse_depth_fwd': ['fuse_depth_fwd_q_k', 'fuse_depth_fwd_k'],
    'fuse_depth_bwd': ['fuse_depth_bwd_gather_k', 'fuse_depth_combine_k', 'fuse_depth_bwd_k', 'fuse_depth_reduce_k'],
    'fuse_pose_fwd': ['fuse_pose_fwd_k'],
    'fuse_pose_bwd': ['pose_fold_k', 'fuse_pose_bwd_k', 'pose_combine_k'],
    'voxel_project_fwd': ['voxel_project_fwd_k'],
    'voxel_project_plan': ['vpb_count_k', 'vpb_scan1_k', 'vpb_scan2_k', 'vpb_fill_k', 'vpb_order_k', 'vpb_tile_k',
                           'vpb_tasks_k'],
    'voxel_project_bwd': ['vpb_fold_zero_k', 'vpb_main_k'],
    'view_stats': ['view_stats_k', 'view_finalize_k'],
    'view_apply': ['view_apply_k'],
    'view_bwd': ['view_bwd_k', 'view_bwd_reduce_k'],
    'photo_fwd': ['photo_fwd_k', 'photo_finalize_k'],
    'photo_bwd': ['photo_bwd_k'],
    'smooth_fwd': ['smooth_fwd_k', 'smooth_finalize_k'],
    'smooth_bwd': ['smooth_bwd_k'],
    'aggregate': ['aggregate_fwd_k', 'aggregate_plane_fwd_k'],
    'proj_conv_fwd': ['pcv_main_k', 'pcvb_main_k', 'pcv_reduce_k'],
    'proj_conv_dgrad': ['pcd_main_k', 'pcd_reduce_k', 'pcdf_main_k', 'pcdf_reduce_k', 'pcg_main_k', 'pcg_reduce_k',
                        'pch_main_k', 'pch_reduce_k'],
    'proj_conv_wgrad': ['pcw_main_k', 'pwb_main_k8', 'pcw_reduce_k', 'pcw_bias_k', 'pwb_bias_k', 'pcw_bias_fin_k'],
    'pad_conv_fwd': ['ppc_main_k', 'ppcb_main_k', 'ppc_reduce_k'],
    'pad_conv_dgrad': ['ppd_main_k', 'ppd_reduce_k'],
    'pad_conv_wgrad': ['pwb_main_k4', 'pwb_reduce_map_k'],
    'depth_syn_fwd': ['depth_syn_fwd_k'],
    'depth_syn_bwd': ['depth_syn_bwd_k'],
    'bn_fwd': ['bn_stats_k', 'bn_sum_k', 'bn_apply_k', 'bn1_fwd_k', 'bn_stats_nhwc_k', 'bn_sum_blk_k', 'bn_apply_nhwc_k'],
    'bn_bwd': ['bn_bwd_stats_k', 'bn_bwd_apply_k', 'bn1_bwd_k', 'bn_bwd_stats_nhwc_k', 'bn_bwd_apply_nhwc_k'],
    'reflect_pad': ['reflect_pad_fwd_k', 'reflect_pad_bwd_k', 'lrelu_pad_bwd_nhwc_k'],
    'upsample_bwd': ['up_ac_bwd_x_k', 'up_ac_bwd_y_k', 'aggregate_plane_bwd_k'],
    'maxpool': ['maxpool_fwd_k', 'maxpool_fwd4_k', 'maxpool_bwd_k', 'maxpool_nhwc_fwd_k', 'maxpool_nhwc_bwd_k'],
    'elu_pad': ['elu_up_pad_fwd_k', 'elu_up_pad_bwd_k'],
    'disp_conv': ['disp_conv_fwd_k', 'disp_conv_dgrad_k', 'disp_conv_wgrad_k'],
    'dec_conv': ['dconv_fwd_k', 'dconv_dgrad_k', 'dconv_wgrad_k'],
}
# Ops timed as several separate C-ABI calls (one ProfScope each, the bench's launch unit): the
# traffic is per call of any of these kernels, not per launch of the first one.
ENTRY = {
    'aggregate': ['aggregate_fwd_k', 'aggregate_plane_fwd_k'],
    'bn_fwd': ['bn_stats_k', 'bn_apply_k', 'bn1_fwd_k', 'bn_stats_nhwc_k', 'bn_apply_nhwc_k'],
    'bn_bwd': ['bn_bwd_stats_k', 'bn_bwd_apply_k', 'bn1_bwd_k', 'bn_bwd_stats_nhwc_k', 'bn_bwd_apply_nhwc_k'],
    'upsample_bwd': ['up_ac_bwd_x_k', 'aggregate_plane_bwd_k'],
    'elu_pad': ['elu_up_pad_fwd_k', 'elu_up_pad_bwd_k'],
    'disp_conv': ['disp_conv_fwd_k', 'disp_conv_dgrad_k'],
    'dec_conv': ['dconv_fwd_k', 'dconv_dgrad_k'],
    'reflect_pad': ['reflect_pad_fwd_k', 'reflect_pad_bwd_k', 'lrelu_pad_bwd_nhwc_k'],
    'maxpool': ['maxpool_fwd_k', 'maxpool_fwd4_k', 'maxpool_bwd_k', 'maxpool_nhwc_fwd_k', 'maxpool_nhwc_bwd_k'],
}


def kernel_of(name):
    """vfd kernel base name from a demangled ('vfd::bn_apply_k<float>(...)') or, as rocprofv3
    leaves the bf16 template instances, mangled ('_ZN3vfd10bn_apply_kIDF16bEEv...') name.  The bf16
    weight-gradient kernel serves two ops: K3C's instance (8 channels per X load) is
    'pwb_main_k8', K2C's (4: the pose map) 'pwb_main_k4'."""
    base = None
    m = re.search(r'vfd::(\w+)', name)
    if m:
        base = m.group(1)
    else:
        m = re.match(r'_ZN3vfd(\d+)', name)
        if m:
            n = int(m.group(1))
            base = name[m.end():m.end() + n]
    if base == 'pwb_main_k':
        base += '8' if ('Li8E' in name or ', 8>' in name) else '4'
    return base


def load(path, counter):
    per = collections.defaultdict(list)
    for r in csv.DictReader(open(path)):
        if r['Counter_Name'] != counter:
            continue
        k = kernel_of(r['Kernel_Name'])
        if k:
            per[k].append(float(r['Counter_Value']))
    return per


def main():
    fetch = load(sys.argv[1], 'FETCH_SIZE')
    write = load(sys.argv[2], 'WRITE_SIZE')
    out = {'_meta': {'unit': 'bytes per op launch', 'fetch_correction': 2.0,
                     'source': 'rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE, separate passes'}}
    for op, ks in OPS.items():
        ks = [k for k in ks if k in fetch]          # kernels this build actually launches
        entry = ENTRY.get(op, ks[:1])
        n = sum(len(fetch.get(k, [])) for k in entry)
        if not n:
            continue
        f = sum(sum(fetch.get(k, [])) for k in ks) / n
        w = sum(sum(write.get(k, [])) for k in ks) / max(sum(len(write.get(k, [])) for k in entry), 1)
        out[op] = round((2.0 * f + w) * 1024)
        out['_meta'][op] = {'fetch_kib': round(f, 1), 'write_kib': round(w, 1), 'launches': n}
    json.dump(out, sys.stdout, indent=1)
    print()


if __name__ == '__main__':
    main()
