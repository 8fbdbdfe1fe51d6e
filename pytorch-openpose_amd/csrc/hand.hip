// hand.hip — placeholder until the hand post path lands
