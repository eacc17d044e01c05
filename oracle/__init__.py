"""CPU oracle for the CGL-GAN per-worker GAN step -- TEST INFRASTRUCTURE ONLY.

This package restates, on torch-CPU, the arithmetic of the reference's hot path
(NetworkCommunication/CGL-GAN: model/mnist_model.py, capgan.py, mixed-gan.py,
CGLGAN/2DMG/*, MDGAN/MNIST/*).  It is the checker the parity tests compare the
HIP path against.  Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s
``cpu_baseline`` leg may import it.  The product path (``cgl-gan_amd/``) never
imports, links or falls back to anything in here.

Parity pin: ``tests/golden/make_golden.py`` imports the reference's own model
modules from ``/root/reference`` (in the build container only) and drives them
with a restatement of the reference drivers' step using ``torch.optim``; the
fixtures it writes under ``tests/golden/`` pin this oracle bit-for-bit at one
CPU thread (``tests/test_oracle_golden.py``).  The reference ships no tests and
no golden vectors of its own, so these fixtures are the only pin.
"""
