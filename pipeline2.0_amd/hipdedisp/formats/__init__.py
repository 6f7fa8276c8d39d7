"""File formats on either side of the dedispersion stage: PSRFITS in, rfifind .mask in,
.subNN/.sub.inf between the two prepsubband calls, .dat/.inf out."""
