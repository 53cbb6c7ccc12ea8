"""Bonus engine: YAML rule DSL, eligibility, awards with the risk abuse check, wagering."""
