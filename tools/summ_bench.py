"""One-screen summary of a bench.py JSON line (headline + nested paths)."""
import json
import sys

d = json.load(open(sys.argv[1]))


def line(name, f):
    r = f['roofline']
    print(f"{name:18s} {f['value']:9.0f} samples/s  {f['ms_per_step']:7.2f} ms/step  whole-step frac "
          f"{f['whole_step_frac_of_peak']:.3f}  FFN1 {r['avg_launch_ms'] * 1e3:6.0f} us live frac {r['frac']:.3f} "
          f"iso {r.get('frac_isolated') or 0:.3f}  [{r['kernel'][:60]}]")
    par = f.get('parity', {})
    print('   parity ' + ', '.join(f"{m} {v['probs_max_abs_err']:.2g} {v['argmax_agree']} risk {v['at_risk_rows']}"
                                   for m, v in par.items() if isinstance(v, dict) and 'probs_max_abs_err' in v))
    pc = f.get('per_config')
    if pc:
        print('   per_config ms ' + ', '.join(f"{k} {v['ms_per_batch']:.3f}" for k, v in pc.items()))


line(d.get('precision', 'headline'), d)
for k in ('fp32_exact_path', 'f16_fast_path', 'fp32x3_path'):
    if k in d:
        line(k, d[k])
if 'cpu_baseline' in d:
    print('cpu_baseline', round(d['cpu_baseline']['value'], 2), d['cpu_baseline']['unit'], 'cores', d['cpu_baseline']['cores'])
