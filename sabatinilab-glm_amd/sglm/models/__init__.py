"""Package layout ``sglm.models`` of the reference (sglm/sglm/models/)."""
