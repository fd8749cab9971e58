"""Mirror of the reference's ``models`` package, restricted to the deformable MSDA path."""
