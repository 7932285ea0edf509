"""Per-(kernel, grid) summary of a rocprofv3 rocpd database."""
import sqlite3
import sys
import glob
import os

path = sys.argv[1]
if os.path.isdir(path):
    path = glob.glob(os.path.join(path, "**", "*.db"), recursive=True)[0]
con = sqlite3.connect(path)
q = """select s.kernel_name, d.grid_size_x/d.workgroup_size_x, d.grid_size_y, d.grid_size_z, count(*),
       avg(d.end-d.start)/1000.0 from rocpd_kernel_dispatch d join rocpd_info_kernel_symbol s
       on d.kernel_id = s.id group by s.kernel_name, d.grid_size_x, d.grid_size_y, d.grid_size_z"""
rows = sorted(con.execute(q), key=lambda r: -r[4] * r[5])
tot = sum(r[4] * r[5] for r in rows)
for r in rows[:int(sys.argv[2]) if len(sys.argv) > 2 else 25]:
    name = r[0].split("_GLOBAL__N_1")[-1][:44]
    print(f"{name:46s} blocks=({r[1]},{r[2]},{r[3]}) n={r[4]:5d} avg_us={r[5]:8.2f} tot={r[4]*r[5]:9.1f} {100*r[4]*r[5]/tot:5.1f}%")
a, b, c = next(con.execute("select min(start), max(end), sum(end-start) from rocpd_kernel_dispatch"))
print("span ms", (b - a) / 1e6, "busy ms", c / 1e6)
