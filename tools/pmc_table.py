"""Per-kernel sums of the counters in a rocprofv3 --pmc output directory
(tools/gpu_pmc_env.sh): ratios for the timing-shape pass, per-wave counts for
the instruction pass."""
import collections
import csv
import glob
import sys

v = collections.defaultdict(lambda: collections.defaultdict(float))
for f in glob.glob(sys.argv[1] + '/**/*counter_collection.csv', recursive=True):
    for r in csv.DictReader(open(f)):
        k = r['Kernel_Name'].split('(')[0].replace('void ', '')[:64]
        v[k][r['Counter_Name']] += float(r['Counter_Value'])
for k, c in sorted(v.items()):
    if 'SQ_WAIT_ANY' in c:
        wc = c['SQ_WAVE_CYCLES'] or 1
        print('%-64s wave_cyc %.3g busy %.3g wait_any %.2f wait_inst %.2f active %.2f valu %.2f lds %.2f '
              'sca %.2f bankconf/lds %.2f' % (k, wc, c['SQ_BUSY_CYCLES'], c['SQ_WAIT_ANY'] / wc,
                                              c['SQ_WAIT_INST_ANY'] / wc, c['SQ_ACTIVE_INST_ANY'] / wc,
                                              c['SQ_ACTIVE_INST_VALU'] / wc, c['SQ_ACTIVE_INST_LDS'] / wc,
                                              c.get('SQ_ACTIVE_INST_SCA', 0) / wc,
                                              c.get('SQ_LDS_BANK_CONFLICT', 0) / max(1, c['SQ_ACTIVE_INST_LDS'])))
    else:
        print('%-64s %s' % (k, '  '.join('%s %.4g' % (n.replace('SQ_', '').lower(), x) for n, x in sorted(c.items()))))
