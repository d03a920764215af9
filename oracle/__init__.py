"""CPU oracle of the SwarmACB e-puck step — TEST INFRASTRUCTURE ONLY (see swarm_oracle.h)."""
