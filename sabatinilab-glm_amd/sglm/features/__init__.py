"""Package layout ``sglm.features`` of the reference (sglm/sglm/features/)."""
