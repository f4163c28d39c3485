"""Configuration contract of the hot path (attrs records with the reference's field names and
defaults, so dicts produced by the reference's confs/templates are accepted unchanged)."""
