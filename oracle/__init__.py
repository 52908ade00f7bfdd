"""CPU oracle for the CGNN neural-receiver forward pass -- TEST INFRASTRUCTURE ONLY.

This package is a numpy restatement of the reference's hot path (the trained
TF/Keras CGNN of theshubh007/neural_rx).  It exists
only to *check* the MI355X engine: it may be imported by ``tests/``,
``__graft_entry__.smoke()`` and the ``cpu_baseline`` leg of ``bench.py``, and by
nothing else.  The product package ``neural_rx_amd`` never imports it; the engine
fails loudly when its HIP library is missing instead of falling back to this code.

Pinning:
* weight layout/param counts: reproduced exactly by the pickled Keras weights
  (nrx_architecture.ipynb:295-308 param counts: 28 634 / 49 074 / 7 812 / 8 328);
* sub-stages pinned by golden vectors captured from the reference's own torch
  modules that are semantically correct (``AggregateUserStates``,
  ``ReadoutLLRs``, ``ReadoutChEst``, ``NRPreprocessing._focc_removal``;
  ``tests/golden/make_golden.py``);
* the separable-conv stacks and the full CGNN have no in-repo executable
  reference (TF/Keras/Sionna are absent): parity against the original TF graph is
  *partially unpinned*; those parts are pinned structurally (weights, Keras
  SeparableConv2D semantics) and by invariance/BER tests (tests/test_oracle.py).
"""
