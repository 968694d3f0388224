from .groups import GroupPlan, TrialGroup, setup_ddp_groups, print0, member_groups
