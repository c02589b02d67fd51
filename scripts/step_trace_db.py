import sqlite3, sys
c = sqlite3.connect(sys.argv[1])
rows = c.execute("select name,start,end,grid_x*grid_y*grid_z/(workgroup_x*workgroup_y*workgroup_z) from kernels order by start").fetchall()
idx = [i for i, r in enumerate(rows) if r[0].startswith("sgd_")]
a, b = idx[-3], idx[-2]
tot = 0
for r in rows[a+1:b+1]:
    d = (r[2]-r[1])/1e3; tot += d
    print(f"{d:8.1f} us wgs {r[3]:6d} {r[0][:60]}")
print("kernels", b-a, "sum", round(tot,1), "span", (rows[b][2]-rows[a][2])/1e3)
