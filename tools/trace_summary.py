"""Summarise a rocprofv3 kernel trace (CSV `*_kernel_trace.csv` or rocpd `*_results.db`):
time per kernel family, per GEMM template/grid, and VGPR counts of the GEMM kernels."""
import collections, csv, sqlite3, sys


def rows(path):
    """Yield (name, ms, grid_x, grid_y, grid_z, vgpr, workgroup_x) per dispatch."""
    if path.endswith('.db'):
        c = sqlite3.connect(path)
        for n, d, gx, gy, gz, vg in c.execute(
                "select name, duration, grid_x, grid_y, grid_z, vgpr_count from kernels"):
            yield n, d / 1e6, gx, gy, gz, vg, 256
    else:
        for x in csv.DictReader(open(path)):
            yield (x['Kernel_Name'], (int(x['End_Timestamp']) - int(x['Start_Timestamp'])) / 1e6,
                   int(x['Grid_Size_X']), int(x['Grid_Size_Y']), int(x['Grid_Size_Z']), int(x.get('VGPR_Count', 0) or 0),
                   int(x.get('Workgroup_Size_X', 256) or 256))


def main():
    fam = collections.defaultdict(float)
    g = collections.defaultdict(lambda: [0, 0.0])
    vg = {}
    for n, t, gx, gy, gz, v, wx in rows(sys.argv[1]):
        base = n.replace('void ', '').replace('(anonymous namespace)::', '')
        fam[base.split('(')[0].split('<')[0]] += t
        if any(q in n for q in ('gemm_f32_kernel', 'gemm_x6_kernel', 'gemm_glds_kernel', 'gemm_hb_kernel', 'gemm_gbf_kernel',
                                'gemm_hbx_kernel', 'gemm_hbp_kernel', 'gemm_hbt_kernel')):
            tmpl = base.split("<")[0][5:9] + ":" + n[n.find('<') + 1:n.find('>')]
            k = (tmpl, gx // max(1, wx), gy, gz)  # grid in blocks (workgroups of wx threads)
            g[k][0] += 1
            g[k][1] += t
            vg[tmpl] = v
    tot = sum(fam.values())
    print(f"total kernel ms {tot:.1f}")
    for k, v in sorted(fam.items(), key=lambda kv: -kv[1])[:25]:
        print(f"  {v:9.2f} ms {100*v/tot:5.1f}%  {k}")
    print("GEMM by template/grid:")
    for k, v in sorted(g.items(), key=lambda kv: -kv[1][1])[:int(sys.argv[2]) if len(sys.argv) > 2 else 30]:
        print(f"  {v[1]:9.2f} ms {v[0]:5d} calls {v[1]/v[0]:.4f} ms/call  {k}")
    print("GEMM VGPRs:", {k: v for k, v in vg.items()})


if __name__ == '__main__':
    main()
