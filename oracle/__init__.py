"""CPU oracle for the MI355X CTR hot path — TEST INFRASTRUCTURE ONLY.

Only ``tests/``, ``__graft_entry__.smoke()`` and the ``cpu_baseline`` leg of
``bench.py`` may import anything under ``oracle/``; the product package
``deep_learning_amd`` never does (it fails loudly when its HIP library is
missing instead of falling back here).

Parity status:
  * model math (embedding/FM/MLP/log-loss/TF1-Adam): PARITY UNPINNED against
    the reference itself — the reference is TensorFlow-1.x graph code, TF is
    not installed and cannot be installed, and the reference ships no tests,
    fixtures or golden vectors.  The restatement follows the reference files
    line by line (citations in ``ctr_ref.py``) and its analytic backward is
    cross-checked against torch autograd in ``tests/test_oracle.py``.
  * ``feat_size`` / ``arg_parse``: pinned by importing the reference's own
    pure-Python ``utils/my_utils.py`` in the build container
    (``tests/golden/make_golden.py``).
  * AUC: pinned against ``sklearn.metrics.roc_auc_score`` (the reference's
    own AUC call, ``models/deepfm_pipeline.py:311``).
  * TFRecord framing: pinned by the CRC-32C known-answer test.
"""
