"""Per-kernel summary of rocprofv3 --pmc CSV passes (several pass directories merged by kernel name)."""
import collections
import csv
import sys


def short(name):
    return name.replace('uda::gpu::', '').replace('(anonymous namespace)::', '').replace('void ', '').split('(')[0]


def load(dirs):
    tot = collections.defaultdict(lambda: collections.defaultdict(float))
    meta = {}
    for d in dirs:
        seen = collections.defaultdict(float)
        for r in csv.DictReader(open(f'{d}/run_counter_collection.csv')):
            k = short(r['Kernel_Name'])
            seen[(k, r['Counter_Name'])] += float(r['Counter_Value'])
            meta[k] = dict(vgpr=r['VGPR_Count'], lds=r['LDS_Block_Size'], wg=r['Workgroup_Size'])
        for (k, c), v in seen.items():
            tot[k][c] = v
    return tot, meta


def row(k, v, m):
    g = v.get
    lds = g('SQ_INSTS_LDS', 0)
    out = [k, m['vgpr'], m['lds']]
    out.append(f"{g('FETCH_SIZE', 0) / 1e6:.2f}" if 'FETCH_SIZE' in v else '-')
    out.append(f"{g('WRITE_SIZE', 0) / 1e6:.2f}" if 'WRITE_SIZE' in v else '-')
    h, mi = g('TCC_HIT_sum'), g('TCC_MISS_sum')
    out.append(f"{h / (h + mi):.2f}" if h is not None and mi is not None and h + mi > 0 else '-')
    out.append(f"{g('SQ_LDS_BANK_CONFLICT', 0) / lds:.2f}" if lds else '-')
    wc = g('SQ_WAVE_CYCLES', 0)
    out.append(f"{100 * g('SQ_WAIT_ANY', 0) / wc:.0f}" if wc else '-')
    out.append(f"{100 * g('SQ_WAIT_INST_LDS', 0) / wc:.0f}" if wc and 'SQ_WAIT_INST_LDS' in v else '-')
    return out


if __name__ == '__main__':
    tot, meta = load(sys.argv[1:])
    print('| kernel | VGPR | LDS B | read GB | write GB | L2 hit | LDS conflict cyc/instr | wait % | wait-LDS-inst % |')
    print('|---|---|---|---|---|---|---|---|---|')
    for k, v in sorted(tot.items(), key=lambda kv: -kv[1].get('SQ_WAVE_CYCLES', 0))[:8]:
        if k.startswith('__amd'):
            continue
        print('| ' + ' | '.join(str(x) for x in row(k, v, meta[k])) + ' |')
