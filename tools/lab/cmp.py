"""Summarise bench lines: value, ms/step, iterations, setup / iteration split."""
import json, sys
for f in sys.argv[1:]:
    d = json.load(open(f))
    c = d.get('config', {})
    print(f"{f.split('/')[-1]:34s} {d['value']/1e6:7.1f} M {d['ms_per_step']:6.3f} ms it={c.get('pcg_iters')} "
          f"setup {c.get('ms_amg_setup', 0):.3f} ms iter {1e3 * c.get('ms_per_pcg_iteration', 0):6.1f} us "
          f"sym {c.get('ms_symbolic', 0):.3f} asm {c.get('ms_assemble', 0):.3f} solve {c.get('ms_solve', 0):.3f}")
