"""Generate tests/golden/cases.json from the pinned Python restatement.

Run from the repo root:  python tests/golden/make_golden.py

Inputs are (a) the content strings of the reference's own tests
(orion-kmer/tests/count_tests.rs:138-141, build_tests.rs, compare_tests.rs),
(b) the reference's fixture files copied byte-for-byte into
tests/golden/data/ (orion-kmer/tests/data/*), and (c) restatement-defined edge
cases (SURVEY.md §8(c) "parity unpinned" list).  Expected outputs come from
oracle/restate.py, which tests/test_oracle_golden.py first checks against
every expectation the reference's tests hold that the reference code can
actually produce (SURVEY.md §4.3 PASS rows), transcribed in
tests/golden/reference_expectations.json.
"""

from __future__ import annotations

import json
import os
import random
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(ROOT, "oracle"))

import restate as R  # noqa: E402

SAMPLE1 = ">seq1\nACGTACGTACGT\n>seq2\nTTTTCCCCGGGGAAAA\n>seq3\nAgCtAgCtNaCcGgTt"
SAMPLE2 = "@read1\nGATTACA\n+\n!!!!!!!\n@read2\nTACATACA\n+\n!!!!!!!!\n@read3\natatatNnN\n+\n!!!!!!!!!"


def text_file(name, content):
    return {"name": name, "text": content}


def data_file(name):
    return {"name": name, "fixture": name}


def load_bytes(f):
    if "text" in f:
        return f["text"].encode()
    with open(os.path.join(HERE, "data", f["fixture"]), "rb") as fh:
        return fh.read()


def rand_seq(rng, n, alphabet="ACGT"):
    return "".join(rng.choice(alphabet) for _ in range(n))


def count_cases():
    rng = random.Random(1234)
    cases = [
        ("ref_sample1_k3", [text_file("sample1.fasta", SAMPLE1)], 3, 1),
        ("ref_sample2_k4", [text_file("sample2.fastq", SAMPLE2)], 4, 1),
        ("ref_both_k5_m2", [text_file("sample1.fasta", SAMPLE1), text_file("sample2.fastq", SAMPLE2)], 5, 2),
        ("ref_sample1_k3_m100", [text_file("sample1.fasta", SAMPLE1)], 3, 100),
        ("fixture1_gz_k7", [data_file("test_input1.fasta.gz")], 7, 1),
        ("fixture1_xz_k7", [data_file("test_input1.fasta.xz")], 7, 1),
        ("fixture1_zst_k7", [data_file("test_input1.fasta.zst")], 7, 1),
        ("fixture2_gz_k6", [data_file("test_input2.fastq.gz")], 6, 1),
        ("fixture2_xz_k6", [data_file("test_input2.fastq.xz")], 6, 1),
        ("fixture2_zst_k6", [data_file("test_input2.fastq.zst")], 6, 1),
        ("fixtures_mixed_k5", [data_file("test_input1.fasta.gz"), data_file("test_input2.fastq.zst")], 5, 1),
        # restatement-defined edge cases
        ("edge_lower_U_gap", [text_file("e.fa", ">a\nacgUuTTga-.~cgtA\n>b\nuuuuACGT\n")], 3, 1),
        ("edge_crlf_multiline", [text_file("e.fa", ">a desc\r\nACGTAC\r\nGTTTGA\r\n>b\r\nGG\r\nCC\r\n")], 4, 1),
        ("edge_short_records", [text_file("e.fa", ">a\nAC\n>b\n\n>c\nACG\n>d\nA\n")], 3, 1),
        ("edge_k1", [text_file("e.fa", ">a\nACGTNNacgt\n")], 1, 1),
        ("edge_k2", [text_file("e.fq", "@r\nAATTCCGG\n+\nIIIIIIII\n")], 2, 1),
        ("edge_k32_polyT", [text_file("e.fa", ">a\n" + "T" * 40 + "\n")], 32, 1),
        ("edge_k32_mixed", [text_file("e.fa", ">a\n" + rand_seq(rng, 300) + "\n>b\n" + rand_seq(rng, 33) + "\n")], 32, 1),
        ("edge_palindrome_k4", [text_file("e.fa", ">a\nGTACGTACGTAC\n")], 4, 1),
        ("edge_all_N", [text_file("e.fa", ">a\nNNNNNNNNNN\n>b\nnnnn\n")], 3, 1),
        ("edge_iupac", [text_file("e.fa", ">a\nACGTRYKMACGTSWBDHVACGT\n")], 3, 1),
        ("edge_spaces_tabs", [text_file("e.fa", ">a\nAC GT\tAC\nGT AC\n")], 5, 1),
        ("edge_headers_only", [text_file("e.fa", ">h1\n>h2\n")], 5, 1),
        ("random_k21", [text_file("r.fa", "".join(f">r{i}\n{rand_seq(rng, rng.randint(10, 200), 'ACGTACGTACGTN')}\n"
                                                  for i in range(60)))], 21, 1),
        ("random_k31_m2", [text_file("r.fq", "".join(f"@r{i}\n{s}\n+\n{'I' * len(s)}\n" for i, s in
                                                      ((i, rand_seq(rng, 150)) for i in range(40))))], 31, 1),
        ("random_k15_dups", [text_file("r.fa", "".join(f">r{i}\n{'ACGTTGCA' * 20}{rand_seq(rng, 30)}\n"
                                                       for i in range(30)))], 15, 2),
    ]
    out = []
    for name, files, k, m in cases:
        tsv = R.run_count_bytes([(f["name"], load_bytes(f)) for f in files], k, m)
        out.append({"name": name, "files": files, "k": k, "min_count": m, "expected_tsv": tsv})
    return out


def build_cases():
    cases = [
        ("ref_build_k3", [text_file("sample1.fasta", SAMPLE1)], 3),
        ("ref_build_dup_k4", [text_file("mini.fasta", ">s1\nACGT\n>s2\nACGT")], 4),
        ("ref_build_multi_k4", [text_file("s1.fa", ">s1\nACGTACGT"), text_file("s2.fa", ">s2\nTACGTACG"),
                                text_file("s3.fa", ">s3\nGGGATCCC")], 4),
        ("ref_build_headers_only_k5", [text_file("no_seq.fa", ">header1\n>header2\n")], 5),
        ("fixture_build_gz_k7", [data_file("test_input1.fasta.gz")], 7),
        ("fixture_build_xz_k6", [data_file("test_input2.fastq.xz")], 6),
    ]
    out = []
    for name, files, k in cases:
        refs = R.build_sets([(f["name"], load_bytes(f)) for f in files], k)
        out.append({"name": name, "files": files, "k": k,
                    "expected": {n: sorted(v) for n, v in refs.items()}})
    return out


def compare_cases():
    db1 = ">seqA\nACGTACGT\n>seqB\nTTTTGGGG"
    db2 = ">seqC\nACGTACGG\n>seqD\nAAAACCCC"
    cases = [
        ("ref_compare_basic_k4", 4, [text_file("db1.fa", db1)], 4, [text_file("db2.fa", db2)]),
        ("ref_compare_identical_k3", 3, [text_file("identical.fa", ">s1\nACGTACGTACGT")], 3,
         [text_file("identical.fa", ">s1\nACGTACGTACGT")]),
        ("ref_compare_no_overlap_k5", 5, [text_file("n1.fa", ">s1\nAAAAACCCCC")], 5, [text_file("n2.fa", ">s2\nTTTTTGGGGG")]),
        ("compare_empty_k5", 5, [text_file("e.fa", ">h\n")], 5, [text_file("f.fa", ">h\n")]),
        ("compare_multi_ref_k4", 4, [text_file("a.fa", db1), text_file("b.fa", db2)], 4, [text_file("c.fa", db2)]),
    ]
    out = []
    for name, k1, f1, k2, f2 in cases:
        r1 = R.build_sets([(f["name"], load_bytes(f)) for f in f1], k1)
        r2 = R.build_sets([(f["name"], load_bytes(f)) for f in f2], k2)
        res = R.compare_sets(k1, r1, k2, r2, "DB1", "DB2")
        out.append({"name": name, "k1": k1, "files1": f1, "k2": k2, "files2": f2, "expected": res,
                    "expected_json": R.compare_json(res)})
    return out


QUERY_READS = ("@read1_match_many\nACGTACGTTT\n+\n!!!!!!!!!!\n@read2_match_one\nTTGCXXXXXX\n+\n!!!!!!!!!!\n"
               "@read3_no_match\nCCCCCCCCCC\n+\n!!!!!!!!!!\n@read4_match_kmer_short_read\nACG\n+\n!!!\n"
               "@read5_match_multiple_hits_but_one_kmer\nACGTACGTACGT\n+\n!!!!!!!!!!!!\n")
QUERY_DB = ">ref_genome_segment\nACGTACGTTTGCATC"


def query_cases():
    """query.rs:24-134.  Output = the matching ids file (placeholder-free)."""
    rng = random.Random(99)
    genome = rand_seq(rng, 3000)
    reads_fq = "".join(f"@q{i} extra words\n{s}\n+\n{'I' * len(s)}\n" for i, s in (
        (i, genome[o:o + 150] if i % 3 else rand_seq(rng, 150))
        for i, o in ((i, rng.randint(0, 2850)) for i in range(50))))
    cases = [
        ("ref_query_basic_k4", 4, [text_file("db.fa", QUERY_DB)], text_file("query_reads.fastq", QUERY_READS), 1),
        ("ref_query_min2_k4", 4, [text_file("db.fa", QUERY_DB)], text_file("query_reads.fastq", QUERY_READS), 2),
        ("ref_query_min8_k4", 4, [text_file("db.fa", QUERY_DB)], text_file("query_reads.fastq", QUERY_READS), 8),
        ("ref_query_min10_k4", 4, [text_file("db.fa", QUERY_DB)], text_file("query_reads.fastq", QUERY_READS), 10),
        ("query_min0_keeps_zero_hit_reads", 4, [text_file("db.fa", QUERY_DB)],
         text_file("query_reads.fastq", QUERY_READS), 0),
        # restatement-defined: no normalize on this path (query.rs:66)
        ("query_raw_lower_U_multiline", 4, [text_file("db.fa", QUERY_DB)],
         text_file("r.fa", ">l lower\nacgtacgttt\n>u has U\nACGUACGTTT\n>m multi\nACG\nTACGTTT\n"
                           ">crlf\r\nACGTAC\r\nGTTTGC\r\n>empty\n>n\nACGTNACGT\n"), 1),
        ("query_fixture_gz_k6", 6, [data_file("test_input2.fastq.xz")], data_file("test_input2.fastq.gz"), 1),
        ("query_fixture_fasta_zst_k5", 5, [data_file("test_input1.fasta.gz")], data_file("test_input1.fasta.zst"), 2),
        ("query_random_k31", 31, [text_file("g1.fa", ">g1\n" + genome[:1500]), text_file("g2.fa", ">g2\n" + genome[1400:])],
         text_file("reads.fastq", reads_fq), 1),
        ("query_random_k31_min60", 31, [text_file("g.fa", ">g\n" + genome)], text_file("reads.fastq", reads_fq), 60),
        ("query_random_k21_min0", 21, [text_file("g.fa", ">g\n" + genome[:500])], text_file("reads.fastq", reads_fq), 0),
    ]
    out = []
    for name, k, dbf, reads, mh in cases:
        refs = R.build_sets([(f["name"], load_bytes(f)) for f in dbf], k)
        res = R.run_query_bytes(k, refs, reads["name"], load_bytes(reads), mh)
        out.append({"name": name, "k": k, "db_files": dbf, "reads": reads, "min_hits": mh,
                    "expected_output": res.decode()})
    return out


CL_INPUT = ">input_seq1\nACGTACGT\n>input_seq2\nACGTACGT\n>input_seq3\nTTTTGGGG"
CL_A = ">db1_refA\nACGTACGTACGT"
CL_B = ">db1_refB\nGGGAAAAATTTT"
CL_C = ">db2_refC\nACGTTACGTT"


def classify_cases():
    """classify.rs:58-385.  JSON/TSV carry the placeholder paths INPUT and
    DB<i>; tests substitute the real paths."""
    rng = random.Random(7)
    genome = rand_seq(rng, 4000)
    reads = "".join(f"@r{i}\n{genome[o:o + 100]}\n+\n{'I' * 100}\n"
                    for i, o in ((i, rng.randint(0, 3900)) for i in range(200)))
    cases = [
        ("ref_classify_basic_k4", text_file("input.fa", CL_INPUT),
         [[text_file("db1_refA.fa", CL_A), text_file("db1_refB.fa", CL_B)], [text_file("db2_refC.fa", CL_C)]], 4, 1, 0.0),
        ("ref_classify_minfreq2_k4", text_file("input.fa", ">S1\nACGTACGT\n>S2\nACGTGGGG"),
         [[text_file("db_ref.fa", CL_A)]], 4, 2, 0.0),
        ("ref_classify_mincov05_k4", text_file("input.fa", CL_INPUT),
         [[text_file("db_refA.fa", CL_A), text_file("db_refB.fa", CL_B)]], 4, 1, 0.5),
        ("ref_classify_mincov01_k4", text_file("input.fa", CL_INPUT),
         [[text_file("db_refA.fa", CL_A), text_file("db_refB.fa", CL_B)]], None, 1, 0.1),
        ("classify_empty_reference_k4", text_file("input.fa", CL_INPUT),
         [[text_file("empty.fa", ">nothing\n"), text_file("db1_refA.fa", CL_A)]], None, 1, 0.0),
        ("classify_no_match_k5", text_file("input.fq", "@r\nAAAAAAAAAA\n+\nIIIIIIIIII\n"),
         [[text_file("c.fa", ">c\nCGCGCGCGTA")]], 5, 1, 0.0),
        ("classify_fixture_gz_input_k5", data_file("test_input1.fasta.gz"),
         [[data_file("test_input2.fastq.gz")]], 5, 1, 0.0),
        ("classify_random_reads_k21", text_file("reads.fq", reads),
         [[text_file("g1.fa", ">g1\n" + genome[:2000]), text_file("g2.fa", ">g2\n" + genome[1800:]),
           text_file("other.fa", ">o\n" + rand_seq(rng, 1000))],
          [text_file("g.fa", ">g\n" + genome)]], 21, 2, 0.3),
    ]
    out = []
    for name, inp, dbs, uk, mf, mc in cases:
        k = uk or 4 if name != "classify_random_reads_k21" else 21
        dbl = []
        for i, files in enumerate(dbs):
            refs = R.build_sets([(f["name"], load_bytes(f)) for f in files], k)
            dbl.append((f"DB{i}", k, [(f["name"], refs[f["name"]]) for f in files]))
        js, tsv = R.run_classify_bytes("INPUT", load_bytes(inp), dbl, uk, mf, mc)
        out.append({"name": name, "input": inp, "k": k, "dbs": dbs, "user_k": uk, "min_freq": mf, "min_cov": mc,
                    "expected_json": js, "expected_tsv": tsv})
    return out


def main():
    doc = {
        "generator": "tests/golden/make_golden.py (oracle/restate.py)",
        "count": count_cases(),
        "build": build_cases(),
        "compare": compare_cases(),
        "query": query_cases(),
        "classify": classify_cases(),
    }
    with open(os.path.join(HERE, "cases.json"), "w") as fh:
        json.dump(doc, fh, indent=1, sort_keys=False)
        fh.write("\n")
    print(f"wrote {len(doc['count'])} count, {len(doc['build'])} build, {len(doc['compare'])} compare, "
          f"{len(doc['query'])} query, {len(doc['classify'])} classify cases")


if __name__ == "__main__":
    main()
