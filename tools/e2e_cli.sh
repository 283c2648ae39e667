#!/bin/bash
# End-to-end CLI wall time on the C2 input (host parse + H2D + count + TSV
# write), reported beside bench.py's device-resident number (SURVEY §8(d)
# "End-to-end ... reported separately").  Inputs live in /tmp on the box.
set -eo pipefail
ROOT=$(cd "$(dirname "$0")/.." && pwd)
CLI=$ROOT/orion-kmer_amd/build/orion-kmer
D=${TMPDIR:-/tmp}/okm_e2e
mkdir -p "$D"
python3 "$ROOT/tools/make_c2_fastq.py" "$D/c2.fastq"
gzip -1 -c "$D/c2.fastq" > "$D/c2.fastq.gz"
ls -la "$D"
TIMEFORMAT="e2e %R s"
run() {
    echo "== $*"
    time timeout -k 10 300 "$CLI" "$@"
}
cat "$D/c2.fastq" > /dev/null
# five plain runs (the first to a fresh file, then over it): the box's I/O
# and CPU share vary run to run, so the median is the number to quote
for i in 1 2 3 4 5; do
    OKM_PROFILE_HOST=1 run count -k 31 -i "$D/c2.fastq" -o "$D/out.tsv" 2>&1 | tee -a "$D/plain.txt"
done
python3 -c "import re,statistics,sys; v=[float(x) for x in re.findall(r'e2e ([0-9.]+) s', open(sys.argv[1]).read())]; print('plain runs', v, 'median', statistics.median(v), 'best', min(v))" "$D/plain.txt"
OKM_PROFILE_HOST=1 run count -k 31 -i "$D/c2.fastq" -o "$D/out2.tsv" -m 2
run count -k 31 -i "$D/c2.fastq.gz" -o "$D/out.tsv.gz"
# the two halves of that run apart: gzip input to a plain table (three runs with
# the single member inflated on the host threads, okm_inflate.cpp, then one
# with the serial libdeflate inflate it replaced), plain input to a gzip table
for i in 1 2 3; do
    OKM_PROFILE_HOST=1 run count -k 31 -i "$D/c2.fastq.gz" -o "$D/out_gzin.tsv"
done
OKM_PROFILE_HOST=1 OKM_GZ_PARALLEL=0 run count -k 31 -i "$D/c2.fastq.gz" -o "$D/out_gzin_serial.tsv"
OKM_PROFILE_HOST=1 run count -k 31 -i "$D/c2.fastq" -o "$D/out_gzout.tsv.gz"
run -v count -k 31 -i "$D/c2.fastq" -o "$D/out.tsv"
wc -l "$D/out.tsv" "$D/out2.tsv"
cmp "$D/out.tsv" <(zcat "$D/out.tsv.gz") && echo "gz output identical"
cmp "$D/out.tsv" "$D/out_gzin.tsv" && cmp "$D/out.tsv" "$D/out_gzin_serial.tsv" && echo "gz input tables identical"
rm -rf "$D"
