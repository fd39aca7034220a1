"""Experiment drivers: DSS/TSS simulation, collaborative vs non-collaborative
training, WMD between models, corpus preprocessing (reference experiments/ and
aux_scripts/)."""
