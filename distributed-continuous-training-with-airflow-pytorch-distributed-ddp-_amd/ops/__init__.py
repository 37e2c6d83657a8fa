"""HIP kernel wrappers (host-side validation + launch) and their CPU/torch references."""
