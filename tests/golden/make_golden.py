"""Generate tests/golden/*.json from the reference's own JUnit known answers.

Every value below is transcribed from an assertion in the reference test tree
(align/src/test/java/org/utgenome/weaver/align/, cited per case as T/<file>:<line>).
The reference cannot be compiled or run here (no JDK, unvendored deps: SURVEY.md
§8c), so these assertions are the pinning vectors for the CPU oracle and, through
it, for the HIP path.  Run:  python tests/golden/make_golden.py
"""
import json
import os

HERE = os.path.dirname(os.path.abspath(__file__))

COMP = {"A": "T", "C": "G", "G": "C", "T": "A", "N": "N"}


def revcomp(s):
    # ACGTSequence.reverseComplement (A/ACGTSequence.java:371-379) on plain ACGTN text
    return "".join(COMP[c] for c in reversed(s))


def bsf_cases():
    """T/strategy/BidirectionalSuffixFilterTest.java: ref AAGCCTAGTTTCCTTG, config.k = 2 (:47-52)."""
    F, R = 0, 1
    cases = [
        # name, query, expected fields (only those the JUnit test asserts), file:line
        ("oneMismatchAtTail", "GCCTAC", dict(cigar="5M1S", start=3, strand=F, nm=0), 69),
        ("oneMismatch", "GCCAAGTT", dict(cigar="8M", start=3, strand=F, nm=1), 78),
        ("oneMismatchReverse", revcomp("GCGTAGTT"), dict(cigar="8M", start=3, strand=R, nm=1), 90),
        ("bidirectionalSearch", "AACCCTAGTTTCGTT", dict(cigar="15M", start=1, strand=F, nm=2), 99),
        ("bidirectionalSearchReverse", revcomp("AACCCTAGTTTCGTT"), dict(cigar="15M", start=1, strand=R, nm=2), 108),
        ("twoMismatchAtHead", "TTGCCTAGTTT", dict(cigar="2S9M", start=3, strand=F, nm=0), 117),
        ("forwardExact", "GCCTAGT", dict(cigar="7M", start=3, strand=F, nm=0), 126),
        ("reverseExact", revcomp("GCCTAGT"), dict(cigar="7M", start=3, strand=R, nm=0), 135),
        ("splitExact", "AAGCCTATCCTTG",
         dict(cigar="7M", start=1, strand=F, nm=0, split=dict(cigar="6M", start=11, strand=F, nm=0)), 144),
        ("splitExactReverse", revcomp("AAGCCTATCCTTG"),
         dict(cigar="7M", start=1, strand=R, nm=0, split=dict(cigar="6M", start=11, strand=R, nm=0)), 160),
        ("longRead", "AAGCCTAGATTCCGTG", dict(start=1, strand=F, nm=2, cigar="16M"), 181),
        ("clip", "AAGCCTAGTTAAAAAA", dict(start=1, end=11, cigar="10M6S"), 190),
        ("clip2", "TTTTTTGAGTTTCCTTG", dict(start=7, end=16, cigar="7S10M"), 201),
        ("oneDeletion", "AAGCCTGTTT", dict(start=1, strand=F, nm=1, cigar="6M1D4M"), 212),
        ("oneInsertion", "AAGCCTCAGTT", dict(start=1, strand=F, nm=1, cigar="6M1I4M"), 223),
        ("twoInsertion", "AAGCCAATAGTTT", dict(start=1, strand=F, nm=2, cigar="5M2I6M"), 234),
    ]
    # Assertion sets that the literal restatement does not reproduce.  The JUnit
    # outcome on the reference itself is unknown (no JVM anywhere in this pipeline).
    #  * clip2: end=16 with start=7 and cigar 7S10M fits none of AlignmentRecord.convert's
    #    branches (end = pos+matchLength, pos+unclipped(cigar)=17, or pos+m=24;
    #    R/AlignmentRecord.java:203-273), so the assertion set cannot hold as written.
    #  * twoInsertion: two insertions need the NFA to advance its active row, but
    #    ReadAlignmentNFA.removeLayersFromAutomaton returns the *previous* automaton when no
    #    layer is trimmed (S/ReadAlignmentNFA.java:205-207), which pins the diagonal states;
    #    the read-end match bit mPos=k+m-progress (:188) is then unreachable.
    unreproduced = {
        "clip2": "assertion set inconsistent with every AlignmentRecord.convert branch (R/AlignmentRecord.java:203-273)",
        "twoInsertion": "unreachable under ReadAlignmentNFA.removeLayersFromAutomaton returning the old automaton "
                        "(S/ReadAlignmentNFA.java:205-207)",
    }
    out = []
    for name, q, exp, line in cases:
        out.append(dict(name=name, query=q, expect=exp, source="T/strategy/BidirectionalSuffixFilterTest.java:%d" % line,
                        unreproduced=unreproduced.get(name)))
    return dict(reference="AAGCCTAGTTTCCTTG", k=2, cases=out)


def bpsw_cases():
    """T/BitParallelSmithWatermanTest.java alignBlockDetailed known answers."""
    cases = [
        ("deletion", "TATACCAAGATCTAGAGATCTGG", "TACCAAGATAGAGATCTGG", 31, 2, "8M2D11M", 2, 184),
        ("mismatches", "GATCTA", "GCTATA", 31, 0, "6M", 2, 194),
        ("insertion", "TATACCAAGATCTAGAGATCTGG", "TACCAAGATCTCTAGAGATCTGG", 31, 2, "8M2I13M", 2, 203),
        ("local", "TATACCAAGATCTAGAGATCTGG", "ACCAAGATCTAGAG", 31, 3, "14M", 0, 213),
        ("softClip2", "TATACCAAGATCTAGAGATCTGG", "GGCGCACCAAGATCTAGAG", 31, 3, "5S14M", 0, 223),
        ("tailClip", "TATACCAAGATCTAGAGTCTGG", "ACCAAGATCTAGAGAAAA", 31, 3, "14M4S", 0, 233),
        ("noMismatch",
         "GCTTCAGTTTCCTGACACTTAAAAAAAAAAGAGTTGCTTATTATTTTAATGAGACTAATGCTTACACTCTGAGTTACTTGTAAGGTGATTGGTTACTTTAATGTTATTATAAGTAATTT",
         "CTGACACTTAAAAAAAAAAGAGTTGCTTATTATTTTAATGAGACTAATGCTTACACTCTGAGTTACTTGTAAGGTGATTGGTTACTTTAATGTTATT",
         11, 11, "97M", 0, 289),
    ]
    out = [dict(name=n, ref=r, query=q, k=k, pos=p, cigar=c, nm=nm,
                source="T/BitParallelSmithWatermanTest.java:%d" % ln) for n, r, q, k, p, c, nm, ln in cases]
    # exactMatch sweep (T/BitParallelSmithWatermanTest.java:304-319): every substring of length
    # 30..len-1 aligns at its own offset with cigar "<len>M" and 0 mismatches (k=2).
    sweep_ref = ("GCTTCAGTTTCCTGACACTTAAAAAAAAAAGAGTTGCTTATTATTTTAATGAGACTAATGCTTACACTCTGAGTTACTTGTAAGGTGATTGGTT"
                 "ACTTTAATGTTATTATAAGTAATTTATTGGTTACTTTAATGTTATTATAAGTAAT")
    return dict(cases=out, exact_sweep=dict(ref=sweep_ref, k=2, min_len=30,
                                            source="T/BitParallelSmithWatermanTest.java:304-319"))


def query_mask_cases():
    """T/QueryMaskTest.java:48-67 mask64: check(query, answer, dir, ch, offset, margin, boundary);
    answer is a BitVector string, LSB rightmost (BitVector.parseString)."""
    # SearchDirection.index: Forward 0, Backward 1 ; ACGT code: A 0
    rows = [
        ("00001011", 0, 0, 0, 0, 59), ("00000101", 0, 1, 0, 0, 60), ("00000001", 0, 3, 0, 3, 61),
        ("00011000", 1, 3, 2, 3, 62), ("00000110", 1, 3, 0, 3, 63), ("00000011", 1, 2, 0, 3, 64),
        ("00000001", 1, 1, 0, 3, 65), ("00000000", 1, 0, 0, 3, 66),
    ]
    out = []
    for ans, d, off, margin, boundary, ln in rows:
        # getBidirectionalPatternMask64(d, offset, boundary, offset, ch, margin) compared on m=8 bits
        out.append(dict(query="AAGATTGC", dir=d, next_idx=off, pivot=boundary, cursor=off, ch=0, margin=margin,
                        expect=int(ans, 2), bits=8, source="T/QueryMaskTest.java:%d" % ln))
    return out


def fm_backward_search_cases():
    """T/FMIndexOnOccTableTest.java:41-69: test.fa (TATAATAATATAATA), BWT of the forward text,
    Occ window 32, successive backwardSearch from [0, N-1)."""
    steps = [("T", 9, 15, 52), ("A", 3, 9, 56), ("T", 12, 15, 60), ("A", 6, 9, 64), ("A", 1, 3, 68)]
    return dict(fasta="fixtures/test.fa", window=32, start=[0, "N-1"],
                steps=[dict(ch=c, lb=lb, ub=ub, source="T/FMIndexOnOccTableTest.java:%d" % ln) for c, lb, ub, ln in steps])


def cyclic_sa_cases():
    """T/sais/CyclicSAISTest.java: cyclic SA answers (texts carry their own smallest sentinel)."""
    mm = "mmiissiissiippii"
    tata = "TATAATAATATAATA"
    return [
        dict(name="sais", text=[ord(c) for c in mm] + [0],
             expect=[16, 15, 14, 10, 6, 2, 11, 7, 3, 1, 0, 13, 12, 9, 5, 8, 4], source="T/sais/CyclicSAISTest.java:45-52"),
        dict(name="saisInt", text=[3, 2, 2, 3, 1, 0], expect=[5, 4, 1, 2, 3, 0], source="T/sais/CyclicSAISTest.java:68-79"),
        dict(name="saisTATA", text=[{"A": 1, "T": 2}[c] for c in tata] + [0],
             expect=[15, 14, 11, 3, 6, 12, 9, 1, 4, 7, 13, 10, 2, 5, 8, 0], source="T/sais/CyclicSAISTest.java:82-90"),
    ]


def misc_cases():
    return dict(
        cigar_merge=[dict(a="12S", b="2S62M", expect="14S62M", source="T/CIGARTest.java:34-40")],
        fast_count=[
            dict(seq="TTTTATTAAAAAAAA", ch=0, s=0, e=15, expect=9, source="T/ACGTSequenceTest.java:210-214"),
            dict(seq="A" * 64, ch=4, s=0, e=64, expect=0, source="T/ACGTSequenceTest.java:341-345"),
            dict(seq="A" * 64, ch=0, s=0, e=64, expect=64, source="T/ACGTSequenceTest.java:347-349"),
        ],
        # BWAlignTest.align3 (T/BWAlignTest.java:78-94): CLI-built index of test2.fa, default
        # config (k = floor(8*0.1f) = 0, -m bsf), query TAAAGTAT -> seq2, REVERSE, start 9, end 17
        bwalign3=dict(fasta="fixtures/test2.fa", query="TAAAGTAT", chr="seq2", strand=1, start=9, end=17,
                      source="T/BWAlignTest.java:78-94"),
        # ReadSequenceReaderTest (T/record/ReadSequenceReaderTest.java:38-76)
        fastq_count=dict(file="fixtures/sample.fastq", count=3, source="T/record/ReadSequenceReaderTest.java:38-55"),
        fasta_reads_count=dict(file="fixtures/reads_sample.fa", count=2, source="T/record/ReadSequenceReaderTest.java:57-76"),
    )


def main():
    data = dict(bsf=bsf_cases(), bpsw=bpsw_cases(), query_mask=query_mask_cases(),
                fm_backward_search=fm_backward_search_cases(), cyclic_sa=cyclic_sa_cases(), misc=misc_cases())
    with open(os.path.join(HERE, "reference_known_answers.json"), "w") as f:
        json.dump(data, f, indent=1)
    print("wrote", os.path.join(HERE, "reference_known_answers.json"))


if __name__ == "__main__":
    main()
