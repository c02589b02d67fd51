"""Per-category kernel time of ONE steady-state training step from a rocprofv3 SQLite db.

usage: python scripts/step_categories.py run_results.db [marker_kernel_prefix]
The step is the span between the last-but-two and last-but-one launches of the optimizer kernel
(default ``sgd_kernel``; ``adam_kernel`` for the LLaMA / DCGAN benches).
"""
import sqlite3, sys, collections
c = sqlite3.connect(sys.argv[1])
rows = c.execute("select name,start,end,grid_x*grid_y*grid_z/(workgroup_x*workgroup_y*workgroup_z) from kernels order by start").fetchall()
marker = sys.argv[2] if len(sys.argv) > 2 else "sgd_kernel"
idx = [i for i, r in enumerate(rows) if r[0].startswith(marker)]
a, b = idx[-3], idx[-2]
cat = collections.defaultdict(lambda: [0,0.0])
for r in rows[a+1:b+1]:
    n = r[0]
    if n.startswith("void conv_igemm_kernel<"):
        k = "conv mode " + n.split("<")[1].split(",")[0]
    elif n.startswith("void conv_pair_kernel<"):
        k = "conv pair (dgrad+wgrad)"
    else:
        k = n.split("(")[0][:50]
    cat[k][0]+=1; cat[k][1]+=(r[2]-r[1])/1e3
tot=sum(v[1] for v in cat.values())
for k,v in sorted(cat.items(), key=lambda x:-x[1][1]):
    print(f"{v[1]:8.1f} us {v[0]:4d}  {100*v[1]/tot:5.1f}%  {k}")
print("total", round(tot,1), "span", (rows[b][2]-rows[a][2])/1e3)
