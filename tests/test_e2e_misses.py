"""The bench e2e clusters whose consensus is not the template are local
optima the reference stops at too (VERDICT r03 Next 5;
scripts/explain_misses.py, profiles/r04_e2e_misses.json).

All 54 of the 512 e2e clusters (seed 2024, rank 0) that miss the template
converge through INIT's 'no candidates found' (model.jl:499-526,937-950) at a
consensus C that no single edit improves -- not one of the 8m+4 STAGE_SCORE
proposals of C beats score(C) (model.jl:521) -- and the template scores lower
than C under the model.  So the greedy stage machine of the reference stops
at C as well; no miss points at a host-restatement slip.

This test re-runs one such cluster through the Python stage machine on the
oracle engine and checks the classification (CPU, a few seconds)."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "scripts"))


def test_e2e_miss_is_a_model_optimum():
    import explain_misses
    row = explain_misses.run_cluster(8, 2024, 0)
    assert not row["equal"] and row["converged"]
    assert row["stop"] == "no candidates found in INIT."
    assert row["class"] == "template_scores_lower"
    assert row["score_t"] < row["score_c"]
    assert row["n_better"] == 0 and row["better_in_aln"] == []
    assert row["edit_distance"] == 1


def test_committed_miss_table_has_no_unexplained_rows():
    import json
    d = json.load(open(os.path.join(REPO, "profiles", "r04_e2e_misses.json")))
    assert d["clusters"] == 512 and d["misses"] == len(d["rows"])
    assert set(d["classes"]) <= {"template_scores_lower", "local_optimum:no_single_edit_improves",
                                 "local_optimum:improving_path_edit_not_proposed_by_reads",
                                 "local_optimum:improving_edits_off_path_not_proposed", "score_unchanged_stop"}
    assert "SLIP" not in d["classes"]
