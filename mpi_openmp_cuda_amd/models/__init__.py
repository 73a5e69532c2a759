"""The alignment scoring model: alphabet, groups, fused score table, problem container, oracles."""
