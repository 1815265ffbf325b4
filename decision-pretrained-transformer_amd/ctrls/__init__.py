"""Reference-named module tree (drop-in for the reference's ctrls/)."""
