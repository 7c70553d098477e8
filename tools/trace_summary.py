"""Summarise a rocprofv3 kernel-trace CSV: time per kernel family and per GEMM grid."""
import collections, csv, sys
r = list(csv.DictReader(open(sys.argv[1])))
fam = collections.defaultdict(float); g = collections.defaultdict(lambda: [0, 0.0])
for x in r:
    n = x['Kernel_Name']; t = (int(x['End_Timestamp']) - int(x['Start_Timestamp'])) / 1e6
    base = n.replace('void ', '').replace('(anonymous namespace)::', '')
    fam[base.split('(')[0].split('<')[0]] += t
    if 'gemm_f32_kernel' in n:
        k = (n[n.find('<') + 1:n.find('>')], int(x['Grid_Size_X']) // 256, int(x['Grid_Size_Y']), int(x['Grid_Size_Z']))
        g[k][0] += 1; g[k][1] += t
tot = sum(fam.values())
print(f"total kernel ms {tot:.1f}")
for k, v in sorted(fam.items(), key=lambda kv: -kv[1])[:25]: print(f"  {v:9.2f} ms {100*v/tot:5.1f}%  {k}")
print("GEMM by template/grid:")
for k, v in sorted(g.items(), key=lambda kv: -kv[1][1])[:int(sys.argv[2]) if len(sys.argv) > 2 else 30]:
    print(f"  {v[1]:9.2f} ms {v[0]:5d} calls {v[1]/v[0]:.4f} ms/call  {k}")
