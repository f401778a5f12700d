"""Static instruction census per k_tcn phase from a -DTCN_MARK -DTCN_ONE build (tcn_kernel.h TMARK comments at the phase
points of TPROBE). usage: python tools/isa_phases.py <file.s> <mangled-kernel-substring>
Prints, per phase interval [marker a -> next marker], the count of VALU (incl. packed and lane ops), MFMA, LDS, VMEM,
SALU and waitcnt instructions. Static counts: inner loops (polls, member sums) count once."""
import collections
import re
import sys

sys.path.insert(0, __file__.rsplit('/', 1)[0])
from isa_stats import body_of, classify  # noqa: E402

# the phase that STARTS at each stamp (TPROBE k in tcn_kernel.h), i.e. the code placed between stamp k and the next
NAMES = {0: "conv1d GEMM", 1: "epilogue+GN1 sums", 2: "P1 publish/poll/halo", 3: "dwconv+GN2 sums", 4: "res_out GEMM",
         5: "row/frame sums", 6: "P3 publish", 7: "P3 poll+GN2 fold", 8: "gates", 9: "moment record",
         10: "P4 publish/poll", 11: "GN_a/GN_b finish", 13: "(after the loop: head)", 14: "x' update", 12: "loop end"}


def main(path, key):
    body = body_of(path, key)
    cur, out = None, collections.OrderedDict()
    for line in body.split('\n'):
        t = line.strip()
        m = re.match(r';;TMARK (\d+)', t)
        if m:
            cur = int(m.group(1))
            out.setdefault(cur, collections.Counter())
            continue
        if not t or t.startswith(('.', ';')) or t.endswith(':') or cur is None:
            continue
        out[cur][classify(t.split()[0])] += 1
    tot = collections.Counter()
    print(f"{'after marker':28s} {'valu':>6s} {'pk':>5s} {'lane':>5s} {'mfma':>5s} {'lds':>5s} {'vmem':>5s} {'salu':>5s} {'wait':>5s}")
    for k, c in out.items():
        tot.update(c)
        print(f"{str(k) + ' ' + NAMES.get(k, ''):28s} {c['valu']:6d} {c['valu_pk']:5d} {c['lane']:5d} {c['mfma']:5d} "
              f"{c['lds']:5d} {c['vmem']:5d} {c['salu']:5d} {c['wait']:5d}")
    print(f"{'total':28s} {tot['valu']:6d} {tot['valu_pk']:5d} {tot['lane']:5d} {tot['mfma']:5d} {tot['lds']:5d} "
          f"{tot['vmem']:5d} {tot['salu']:5d} {tot['wait']:5d}")


if __name__ == '__main__':
    main(sys.argv[1], sys.argv[2])
