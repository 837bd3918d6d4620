"""Drop-in DDP comm hooks (same module layout as the reference's ``comm_hooks``)."""
